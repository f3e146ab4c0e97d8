# same-box A/B of two builds: lib/libupr_prev.so (A) vs lib/libupr.so (B) on conv shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-libab}
mkdir -p $out
SH=${SHAPES:-bneck,bneckr,dec3,dec3p,aspp6,aspp18,enc3s2,fuse}
for i in 1 2; do
  echo "A prev" >> $out/bench.txt
  UPR_LIB=$GRAFT_REPO_ROOT/retinex-image-enhancement_amd/lib/libupr_prev.so timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes $SH --iters 30 >> $out/bench.txt 2>&1 || exit $?
  echo "B new" >> $out/bench.txt
  timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes $SH --iters 30 >> $out/bench.txt 2>&1 || exit $?
done
grep -v amdgpu $out/bench.txt
