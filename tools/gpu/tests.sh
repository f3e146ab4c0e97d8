# full -m gpu suite (no -x: every failure reported), then optionally the default bench line
# usage: CK=<dir under gpurun_out> [BENCH=1] bash tools/gpu/tests.sh [pytest selection...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-t}
mkdir -p $out
sel="${@:-tests}"
timeout -k 10 900 python -u -m pytest $sel -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $out/gpu_tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || exit $?
fi
exit $rc
