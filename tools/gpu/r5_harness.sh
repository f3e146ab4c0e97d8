# enhance harness (main.py --mode enhance over a directory): PNG writer-thread count A/B at 256^2 / 512^2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-r5harness}
mkdir -p $out
for w in 6 14 6 14; do
  for s in 256 512; do
    UPR_PNG_WRITERS=$w timeout -k 10 300 python tools/harness_bench.py --n 32 --size $s > $out/h_${w}_${s}.json 2> $out/h_${w}_${s}.err || exit $?
    echo "writers $w size $s $(cat $out/h_${w}_${s}.json)"
  done
done
