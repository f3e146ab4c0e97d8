cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/c3k3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread > $O/train_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --train --amp --steps 5 --warmup 2 --cpu-seconds 0 > $O/train_gather.json 2> $O/train_gather.err || exit 1

