cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/diag
mkdir -p $O
timeout -k 10 200 python -u tools/train_determinism.py 0 1 > $O/det01.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -v -s --timeout 120 --timeout-method thread > $O/train_tests.log 2>&1
echo "rc=$?"
