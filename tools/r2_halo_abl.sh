# halo-tiled wide kernel timing ablations (UPR_HALO_ABL: 0 full, 1 no B DMA, 2 no DMA, 3 no MFMA) + gathered (UPR_WIDE_HALO=0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
for r in 1 2; do
for a in 0 1 2 3; do
echo "abl=$a" >> gpurun_out/abl/cb.log
UPR_HALO_ABL=$a timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,dec3 --iters 30 2>/dev/null >> gpurun_out/abl/cb.log || exit 1
done
echo "gathered" >> gpurun_out/abl/cb.log
UPR_WIDE_HALO=0 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,dec3 --iters 30 2>/dev/null >> gpurun_out/abl/cb.log || exit 1
done
cat gpurun_out/abl/cb.log
