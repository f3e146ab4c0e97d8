# fp32 FAM fusion on the halo kernel: tile rows / occupancy sweep (UPR_HALO) over the fp32 bench breakdown
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/hf32
for cfg in default 4,1 4,2 4,3 8,2; do
  if [ "$cfg" = default ]; then unset UPR_HALO; else export UPR_HALO=$cfg; fi
  timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/hf32/b.json 2> gpurun_out/hf32/b_$cfg.err || exit $?
  echo "$cfg $(python3 -c "import json; d=json.loads(open('gpurun_out/hf32/b.json').read().strip().splitlines()[-1]); print(round(d['value'],1))") $(grep -E 'scale1.2.fusion|scale2.3.fusion' gpurun_out/hf32/b_$cfg.err | awk '{print $1, $3}' | tr '\n' ' ')"
done
