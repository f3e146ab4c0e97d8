# full -m gpu suite + smoke, then convbench on the ring / hwide4 shapes and the fp16 + default bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5f}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes ${SHAPES:-dec1p,dec1,fam_h,fam64,dec2p,dec2,enc1c2,bneck,bneckr,aspp6,dec3p} --iters 30 > $out/convbench.txt 2>&1 || exit $?
grep -v amdgpu.ids $out/convbench.txt
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --no-nested --cpu-seconds 0 --no-traffic --breakdown --detail $out/fp16_detail.json > $out/bench_fp16.json 2> $out/bench_fp16.err || exit $?
python3 -c "import json;d=json.load(open('$out/bench_fp16.json'));print('fp16', d['value'], d['roofline']['frac'], d['roofline']['mfma_bound_layers'], d['roofline']['layer_roofline_frac'])"
