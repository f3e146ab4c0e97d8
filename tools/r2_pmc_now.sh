# fresh PMC passes over one fp16 preact+ASPP forward + per-dispatch table
export PMC_PREC=${PMC_PREC:-fp16} PMC_VARIANT=${PMC_VARIANT:-preact_aspp}
bash tools/pmc_model.sh || exit 1
cd $GRAFT_REPO_ROOT
P=$PMC_PREC
timeout -k 10 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcm_${P}_f -o p --output-format csv -- python3 bench.py --precision $P --variant $PMC_VARIANT --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_${P}_f.log 2>&1 || exit 1
timeout -k 10 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcm_${P}_w -o p --output-format csv -- python3 bench.py --precision $P --variant $PMC_VARIANT --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_${P}_w.log 2>&1 || exit 1
python3 tools/pmc_dispatch.py gpurun_out/pmcm_${P}_a gpurun_out/pmcm_${P}_b gpurun_out/pmcm_${P}_f gpurun_out/pmcm_${P}_w > gpurun_out/pmc_${P}_dispatch.txt 2>&1
cat gpurun_out/pmc_${P}_dispatch.txt
