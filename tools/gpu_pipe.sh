cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "conv2d or fp16 or full_size" > $O/tests.log 2>&1 || exit 1
for k in 0 3; do
UPR_WIDE_KIND=$k timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,aspp6,aspp18,fuse,enc3s2,enc2s2,dec3 --iters 20 > $O/cb_$k.log 2>&1 || exit 1
UPR_WIDE_KIND=$k UPR_WIDE_ABL=3 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,aspp18 --iters 20 > $O/cba_$k.log 2>&1 || exit 1
done
for k in 0 3; do
UPR_WIDE_KIND=$k timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > $O/bd_$k.json 2> $O/bd_$k.err || exit 1
done
