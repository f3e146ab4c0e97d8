# full -m gpu suite + fp16 preact+ASPP per-layer breakdown and bench after a kernel change
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-dsm}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --breakdown --steps 10 > $out/fp16pa.json 2> $out/fp16pa_layers.txt || exit $?
cat $out/fp16pa.json
