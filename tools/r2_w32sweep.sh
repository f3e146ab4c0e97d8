# wide32 tile-config sweep per shape (fp32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/w32s
S128=bneck,enc2s2,enc3s2,dec3,aspp18,fuse,enc2c2,up1,up2,up3
S64=enc1s2,fam_h,dec2,enc1c2
for c in 8 9; do
  UPR_WIDE32=$c timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes $S128 --iters 10 > gpurun_out/w32s/d$c.txt 2>&1 || exit 1
done
for c in 6 7; do
  UPR_WIDE32=$c timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes $S64,$S128 --iters 10 > gpurun_out/w32s/d$c.txt 2>&1 || exit 1
done
for f in gpurun_out/w32s/d*.txt; do echo "== $f"; grep -h fp32 $f; done
