# Same-box A/B of whole forward steps under different env settings, after the forward parity files
# (run under the B env): fp16 preact+ASPP (configs[2]) and fp32 plain (configs[1]), alternating
# A / B (/ C) $ROUNDS times, --no-profile (every timed step on the production path).
#   AENV="UPR_MS_STREAMS=0" BENV="UPR_MS_STREAMS=1" CENV="UPR_MS_PRIO=1" bash tools/gpu/env_ab.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-envab}
mkdir -p $out
env ${BENV:-UPR_X=1} timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bn_parity.py tests/test_gpu_modules.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in $(seq ${ROUNDS:-2}); do
  for side in A B C; do
    if [ $side = A ]; then e="${AENV:-UPR_X=0}"; elif [ $side = B ]; then e="${BENV:-UPR_X=1}"; else e="${CENV:-}"; fi
    [ -z "$e" ] && continue
    env $e timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --no-profile --steps 30 > $out/fp16_$side$i.json 2> $out/fp16_$side$i.err || exit $?
    python3 -c "import json;d=json.load(open('$out/fp16_$side$i.json'));print('$side fp16 $e', round(d['value'],1), round(d['ms_per_step'],4))" | tee -a $out/ab.txt
    env $e timeout -k 10 200 python bench.py --cpu-seconds 0 --no-traffic --no-nested --no-profile --steps 20 > $out/fp32_$side$i.json 2> $out/fp32_$side$i.err || exit $?
    python3 -c "import json;d=json.load(open('$out/fp32_$side$i.json'));print('$side fp32 $e', round(d['value'],1), round(d['ms_per_step'],4))" | tee -a $out/ab.txt
  done
done
