# (the UPR_HW4_W256 switch was removed after this A/B: profiles/r5_hw4_w256_ab.txt)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5w256
mkdir -p $out
UPR_HW4_W256=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv" > $out/tests.log 2>&1; tail -1 $out/tests.log
for v in 0 1 0 1; do
  UPR_HW4_W256=$v timeout -k 10 200 python -u tools/convbench.py --shapes vgg21,enc1c2 --bufs 4 --iters 30 2>&1 | grep -v amdgpu.ids | sed "s/^/W256=$v /"
done
