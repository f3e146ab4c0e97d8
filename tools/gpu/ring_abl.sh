# ring-kernel timing ablations (tools/convbench.py; ablated results are garbage): UPR_RING_ABL=0
# production, 1 = no ring DMA after the first two steps, 2 = no MFMAs; plus the multi-scale re-check
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-ringabl}
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py -k "multiscale" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profE -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh_prof.json 2>&1 || exit $?
for i in 1 2; do
  for a in 0 1 2; do
    echo "ABL=$a" >> $out/abl.txt
    UPR_RING_ABL=$a timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes ${SHAPES:-dec1p,fam_h,dec2p} --iters 30 >> $out/abl.txt 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $out/abl.txt
