cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/red4ab
mkdir -p $O
for v in 1 0 1 0; do
UPR_REDUCE4=$v timeout -k 10 300 python bench.py --train --amp --steps 6 --warmup 2 --cpu-seconds 0 > $O/t_$v.json 2> $O/t_$v.err || exit 1
python -c "import json;d=json.load(open('$O/t_$v.json'));print('$v',d['value'])" >> $O/summary.txt
done
