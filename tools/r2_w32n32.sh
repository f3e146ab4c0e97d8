# fp32 32-wide GEMM at 512^2 (FAM fusion class): halo kernel vs wide32 256x32 / 512x32 tiles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/n32
for n in 0 1 2 3; do
echo "n32=$n" >> gpurun_out/n32/cb.log
UPR_WIDE32_N32=$n timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes fam64 --iters 10 2>/dev/null >> gpurun_out/n32/cb.log || exit 1
done
cat gpurun_out/n32/cb.log
