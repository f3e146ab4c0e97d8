# fp32-output epilogues for the training step's autocast convs: training tests, inference conv parity, AMP bench A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/o32
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/o32/tests.log 2>&1
rc=$?; tail -3 gpurun_out/o32/tests.log; [ $rc -eq 0 ] || exit $rc
for o in 0 1; do
UPR_T_OUT32=$o timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/o32/train_$o.json 2> gpurun_out/o32/train_$o.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/o32/train_$o.json').read().strip().splitlines()[-1]); print('out32=$o train amp', round(d['value'],1), 'img/s', round(d['ms_per_step'],2), 'ms')"
done
