cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/abl
mkdir -p $O
for a in 0 1 2 3; do
UPR_WIDE_KIND=0 UPR_WIDE_ABL=$a timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,aspp18,fuse,enc3s2,dec3 --iters 20 > $O/cb_$a.log 2>&1 || exit 1
done
