# full suite + convbench + fp16 bench (r5_full.sh), pointwise / stride-2 hwide4 A/B, enhance leg with rocprofv3 stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SHAPES=${SHAPES:-dec1p,dec1,fam_h,fam64,dec2p,dec2,enc1c2,bneck,bneckr,aspp6,dec3p,fuse1k,a1x1,enc3s2,enc2s2} bash tools/gpu/r5_full.sh || exit $?
cd $GRAFT_REPO_ROOT
# pointwise hwide4 vs the gathered kernel on the ASPP 1x1 shapes
UPR_HW4_PW=0 UPR_HW4_S2=0 timeout -k 10 120 python tools/convbench.py --dtype fp16 --shapes fuse1k,a1x1,enc3s2,enc2s2 --iters 30 2>&1 | grep -v amdgpu.ids || exit $?
out=gpurun_out/${CK:-r5c}
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/profE -o p --output-format csv -- python3 bench.py --enhance --steps 20 --warmup 3 --no-traffic --cpu-seconds 0 --detail "" > $out/enh_prof.json 2>&1 || exit $?
python3 -c "
import csv,glob
f=glob.glob('$out/profE/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('ms_','clahe','lab','gray')): print(r['Name'][:60], r['Calls'], r['AverageNs'])
"
