cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wide
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "conv2d or fp16 or full_size" > gpurun_out/wide/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/wide/tests.log; [ $rc -le 1 ] || exit 1
for w in 0 1; do
UPR_CONV_WIDE=$w timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,aspp6,aspp18,fuse,enc3s2,enc2s2,dec3 --iters 20 > gpurun_out/wide/cb_$w.log 2>&1 || exit 1
done
for w in 0 1; do
UPR_CONV_WIDE=$w timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/wide/bd_$w.json 2> gpurun_out/wide/bd_$w.err || exit 1
done
