# hwide4 bottleneck-form timing ablations (tools/convbench.py; results of ablated runs are garbage):
# UPR_HW4_ABL=0 production, 16 = no LDS-read drain before each barrier, 48 = no barrier either, 1 = no main-loop DMA
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-hw4abl}
mkdir -p $out
for i in 1 2; do
  for a in 0 16 48 1; do
    echo "ABL=$a" >> $out/abl.txt
    UPR_HW4_ABL=$a timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes ${SHAPES:-bneck,bneckr} --iters 30 >> $out/abl.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/abl.txt
