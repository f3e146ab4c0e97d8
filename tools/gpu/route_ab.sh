# routing A/B after the direct-store epilogues: dilated hwide4 vs gathered+DS on the ASPP shapes,
# hwide4 vs gathered+DS on the bottleneck / dec3 shapes (same box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-routeab}
mkdir -p $out
for i in 1 2; do
  echo "default (hwide4 DL / halo)" >> $out/bench.txt
  timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes aspp6,aspp12,aspp18,bneck,bneckr,dec3,dec3p --iters 30 >> $out/bench.txt 2>&1 || exit $?
  echo "UPR_HW4_DIL=0 UPR_WIDE_HALO=0 (gathered + DS)" >> $out/bench.txt
  UPR_HW4_DIL=0 UPR_WIDE_HALO=0 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes aspp6,aspp12,aspp18,bneck,bneckr,dec3,dec3p --iters 30 >> $out/bench.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $out/bench.txt
