# column-mapped 32 -> 32 ring: conv + model parity, convbench A/B (4 HBM-resident input copies), fp16 layer breakdown
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5col}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 1 0 1 0; do
  echo "COL=$c" >> $out/cb.txt
  UPR_RING_COL=$c timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes dec1p,dec1 --iters 30 --bufs 4 >> $out/cb.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $out/cb.txt
for c in 1 0; do
  UPR_RING_COL=$c timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --no-nested --cpu-seconds 0 --no-traffic --breakdown --detail "" > $out/b16_$c.json 2> $out/b16_$c.err || exit $?
  python3 -c "import json;d=json.load(open('$out/b16_$c.json'));print('COL=$c fp16', d['value'])"
  grep -E "dec1.conv|residual_head" $out/b16_$c.err
done
