cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/w128b
mkdir -p $O
UPR_WIDE128_S1=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "conv2d or fp16 or full_size" > $O/tests.log 2>&1 || exit 1
for v in 0 1 0 1; do
UPR_WIDE128_S1=$v timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > $O/bd_$v.json 2> $O/bd_$v.err || exit 1
python -c "import json;print('$v', json.load(open('$O/bd_$v.json'))['value'])" >> $O/summary.txt
done
