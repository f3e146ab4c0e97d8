# two-chunk shortcut hwide4 (enc3.conv2): full suite + smoke + fp16 bench, then the fp16 layer breakdown with
# the gathered kernel (UPR_HW4_SC2=0) for A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
NO_BENCH= SHAPES=bneck,bneckr bash tools/gpu/r5_full.sh || exit $?
cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5sc2}
UPR_HW4_SC2=0 timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --no-nested --cpu-seconds 0 --no-traffic --breakdown --detail "" > $out/b16_off.json 2> $out/b16_off.err || exit $?
python3 -c "import json;d=json.load(open('$out/b16_off.json'));print('SC2 off fp16', d['value'])"
grep -E "enc3|enc2.conv2" $out/bench_fp16.err $out/b16_off.err
