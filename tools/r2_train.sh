# training GPU tests + train benches (AMP autocast fp16 convs, and fp32)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tr2
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_modules.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tr2/tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|cosine|bs8 512" gpurun_out/tr2/tests.log | tail -45
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/tr2/train_amp.json 2> gpurun_out/tr2/train_amp.err || { tail -5 gpurun_out/tr2/train_amp.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tr2/train_amp.json'));print('amp', d['value'], d['ms_per_step'], d['last_loss']['total'])"
timeout -k 10 300 python bench.py --train --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/tr2/train_fp32.json 2> gpurun_out/tr2/train_fp32.err || { tail -5 gpurun_out/tr2/train_fp32.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/tr2/train_fp32.json'));print('fp32', d['value'], d['ms_per_step'], d['last_loss']['total'])"
