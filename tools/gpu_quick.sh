# quick fp16 check: parity subset + preact_aspp breakdown.  OUT=<dir under gpurun_out>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT:-quick}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k "${TESTK:-conv2d or fp16 or full_size or batch_indep or ienet}" > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log; [ $rc -le 1 ] || exit 1
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > $O/bd_pa.json 2> $O/bd_pa.err || exit 1
