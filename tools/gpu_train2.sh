cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/train2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -v --timeout 200 --timeout-method thread > $O/train_tests.log 2>&1
echo "tests rc=$?" >> $O/train_tests.log
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 10 > $O/train_amp.json 2> $O/train_amp.err
