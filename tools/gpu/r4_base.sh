cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4base
timeout -k 10 200 python bench.py --precision fp16 --variant preact_aspp --cpu-seconds 0 --no-traffic --breakdown --steps 5 > gpurun_out/r4base/fp16pa.json 2> gpurun_out/r4base/fp16pa.err && \
timeout -k 10 200 python tools/convbench.py --dtype fp16 --shapes bneck,bneckr,aspp6,aspp12,aspp18,dec3p,dec3,enc2s2,enc2c2,enc3s2,fuse,fam_h,dec2p --iters 30 > gpurun_out/r4base/convbench.txt 2>&1
