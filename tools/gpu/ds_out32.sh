# direct-store epilogue for the autocast fp32 outputs: training tests + same-box A/B of the configs[4] step
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-dsout32}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes bneck,bneckr,dec3,aspp6 --iters 30 > $out/time.txt 2>&1 || exit $?
grep -v amdgpu $out/time.txt
for i in 1 2; do
  for v in 0 1; do
    UPR_DS_OUT32=$v timeout -k 10 300 python bench.py --train --amp --steps 20 --warmup 3 --no-nested --cpu-seconds 0 > $out/train_$v$i.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('$out/train_$v$i.json'));print('UPR_DS_OUT32=$v train_amp', round(d['value'],1), 'img/s', round(d['ms_per_step'],3), 'ms')" | tee -a $out/ab.txt
  done
done
