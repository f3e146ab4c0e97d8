# hwide4 timing ablations on the bottleneck conv (UPR_HW4_ABL bits: 1 no main-loop DMA, 2 no fragment reads,
# 4 no epilogue, 8 no MFMAs)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4abl}
mkdir -p $out
for a in 0 1 2 3 4 7 8 12 0; do
  echo "ABL=$a" >> $out/bench.txt
  UPR_HW4_ABL=$a timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck --iters 30 >> $out/bench.txt 2>&1 || exit $?
done
cat $out/bench.txt
