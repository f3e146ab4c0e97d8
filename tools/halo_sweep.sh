# UPR_HALO="<tile rows>,<waves per SIMD>" sweep of the halo conv kernel on the UP-Retinex layer shapes
set -e
CFGS=${CFGS:-"4,1 4,2 8,1"}
for cfg in $CFGS; do
  for dt in fp16 fp32; do
    echo "== UPR_HALO=$cfg $dt"
    UPR_HALO=$cfg timeout -k 10 120 python tools/convbench.py --dtype $dt --shapes ${SHAPES:-dec1,fam_h,dec2,dec3,bneck,d2} --iters 20 2>&1 | grep -v amdgpu.ids
  done
done
