# round-2 baseline: fp32 per-layer breakdown + PMC counters of the fp32 conv kernels + default bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2base
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 3 > gpurun_out/r2base/fp32_bd.json 2> gpurun_out/r2base/fp32_bd.err || exit $?
PMC_PREC=fp32 bash tools/pmc_model.sh || exit $?
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcm_fp32_f -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_fp32_f.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcm_fp32_w -o p --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_fp32_w.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r2base/bench_default.json 2> gpurun_out/r2base/bench_default.err
