# event-profiling overhead in the timed region: bench with and without per-launch HIP events
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/povh
for r in 1 2; do
for p in "" "--no-profile"; do
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --steps 20 $p 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fp16 $p', round(d['value'],1), round(d['ms_per_step'],3))" >> gpurun_out/povh/r.log || exit 1
timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --steps 10 $p 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('fp32 $p', round(d['value'],1), round(d['ms_per_step'],3))" >> gpurun_out/povh/r.log || exit 1
done; done
cat gpurun_out/povh/r.log
