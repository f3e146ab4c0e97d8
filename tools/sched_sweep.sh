# UPR_HALO_SCHED experiments: 1 setprio / 2 stagger / 4 no staging / 8 no epilogue
set -e
DEF="0,0 4,0 8,0 12,0"
for sc in ${SCS:-$DEF}; do
  for dt in ${DTS:-fp32 fp16}; do
    echo "== SCHED=$sc $dt"
    UPR_HALO_SCHED=$sc timeout -k 10 120 python tools/convbench.py --dtype $dt --shapes ${SHAPES:-dec1,dec2,bneck} --iters 20 2>&1 | grep -v amdgpu.ids
  done
done
