# same-box A/B of the whole fp16 preact+ASPP step: env A ($AENV) vs env B ($BENV), alternating 3x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${CK:-stepab}
mkdir -p $out
for i in 1 2 3; do
  for side in A B; do
    if [ $side = A ]; then e="$AENV"; else e="$BENV"; fi
    env $e timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --no-nested --steps 20 > $out/$side$i.json 2> $out/$side$i.err || exit $?
    python3 -c "import json;d=json.load(open('$out/$side$i.json'));print('$side', '$e', round(d['value'],1), round(d['ms_per_step'],4))" | tee -a $out/ab.txt
  done
done
