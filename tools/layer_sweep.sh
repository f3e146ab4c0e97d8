# Per-layer times of the whole forward under each UPR_HALO="<th>,<occ>" (bench.py --breakdown);
# CFGS entry "default" = the built-in per-program table
set -e
CFGS=${CFGS:-"4,2 4,3 8,1 8,2"}
for dt in ${DTS:-fp32 fp16}; do
  for cfg in $CFGS; do
    if [ "$cfg" = default ]; then
      timeout -k 10 300 python bench.py --precision $dt --steps 5 --warmup 2 --breakdown --no-traffic --cpu-seconds 0 > gpurun_out/ls_${dt}_0_0.log 2>&1
    else
      UPR_HALO=$cfg timeout -k 10 300 python bench.py --precision $dt --steps 5 --warmup 2 --breakdown --no-traffic --cpu-seconds 0 > gpurun_out/ls_${dt}_${cfg/,/_}.log 2>&1
    fi
  done
done
