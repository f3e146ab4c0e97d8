"""Print the arguments of selected C-ABI calls made during one AMP training
step (bench.py --train --amp), e.g. to see the BN backward flags per layer.
usage: python tools/call_flags.py upr_t_bn_bwd_fused16[,name2...]"""
import os
import runpy
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "retinex-image-enhancement_amd"))
from upr import _lib as L  # noqa: E402

names = sys.argv[1].split(",")
lib = L.lib()
for n in names:
    f = getattr(lib, n)

    def wrap(*a, _f=f, _n=n):
        vals = [getattr(x, "value", x) for x in a]
        where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()[-2:-6:-1])
        print(_n, [v if isinstance(v, int) and abs(v) < 1 << 20 else ("p" if v else 0) for v in vals], where,
              flush=True)
        return _f(*a)
    setattr(lib, n, wrap)
sys.argv = ["bench.py", "--train", "--amp", "--steps", "1", "--warmup", "0", "--cpu-seconds", "0"]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bench.py"), run_name="__main__")
