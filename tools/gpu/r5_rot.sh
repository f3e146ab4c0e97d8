# pointwise hwide4 chunk rotation A/B: convbench over 4 input copies (HBM-resident, as in the model) and the
# fp16 model breakdown, rotation on (default) / off (UPR_HW4_PW=2) / gathered kernel (UPR_HW4_PW=0)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5rot}
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv2d_nhwc" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for m in 1 2 0 1; do
  echo "PW=$m" >> $out/cb.txt
  UPR_HW4_PW=$m UPR_HW4_S2=$([ $m = 0 ] && echo 0 || echo 1) timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes fuse1k,a1x1,enc3s2,enc2s2,bneck,dec2p --iters 24 --bufs 4 >> $out/cb.txt 2>&1 || exit $?
done
grep -v amdgpu.ids $out/cb.txt
for m in 1 2; do
  UPR_HW4_PW=$m timeout -k 10 300 python bench.py --precision fp16 --variant preact_aspp --no-nested --cpu-seconds 0 --no-traffic --breakdown --detail "" > $out/b16_$m.json 2> $out/b16_$m.err || exit $?
  python3 -c "import json;d=json.load(open('$out/b16_$m.json'));print('PW=$m fp16', d['value'])"
  grep -E "fusion|conv1x1|enc3.conv1|enc2.conv1" $out/b16_$m.err | grep -v scale
done
# training: the gradient tests (conv_pw's dense staged epilogue), then the configs[4] step
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/train_tests.log 2>&1
rc=$?; tail -2 $out/train_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --train --amp --steps 10 --warmup 3 --cpu-seconds 0 --detail $out/train_detail.json > $out/train.json 2> $out/train.err || exit $?
python3 -c "import json;d=json.load(open('$out/train.json'));print('train', d['value'], d['ms_per_step'])"
