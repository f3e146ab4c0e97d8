# PMC passes over one fp16 preact+ASPP forward (ring kernels), then summary
export PMC_PREC=fp16 PMC_VARIANT=preact_aspp
bash tools/pmc_model.sh || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcm_fp16_f -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_fp16_f.log 2>&1 || exit 1
timeout -k 10 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcm_fp16_w -o p --output-format csv -- python3 bench.py --precision fp16 --variant preact_aspp --steps 1 --warmup 1 --no-traffic --no-profile --cpu-seconds 0 > gpurun_out/pmcm_fp16_w.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmcm_fp16_a gpurun_out/pmcm_fp16_b gpurun_out/pmcm_fp16_f gpurun_out/pmcm_fp16_w > gpurun_out/pmc16_summary.txt 2>&1
grep -A22 "ring" gpurun_out/pmc16_summary.txt | head -120
