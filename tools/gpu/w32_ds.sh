# fp32 wide kernel direct-store epilogue: parity + same-box A/B (convbench shapes and the configs[1] step)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-w32ds}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 0 1; do
    echo "UPR_WIDE32_DS=$v" >> $out/bench.txt
    UPR_WIDE32_DS=$v timeout -k 10 120 python tools/convbench.py --dtype fp32 --shapes bneck,dec3,dec2,enc3s2,fuse,aspp6 --iters 10 >> $out/bench.txt 2>&1 || exit $?
    UPR_WIDE32_DS=$v timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --no-nested --steps 20 > $out/fp32_$v$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$out/fp32_$v$i.json'));print('configs[1] fp32 step', round(d['value'],1), 'img/s', round(d['ms_per_step'],3), 'ms', 'frac', round(d['roofline']['frac'],4))" >> $out/bench.txt
  done
done
grep -v amdgpu.ids $out/bench.txt
