#!/usr/bin/env python3
"""Per-dispatch PMC table over the LAST forward of separate rocprofv3 --pmc
passes of the same deterministic command (dispatches matched by order).

  python tools/pmc_dispatch.py DIR_a DIR_b [DIR_f DIR_w] [--match conv] [--min-us 20]
"""
import csv
import os
import re
import sys
from collections import OrderedDict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("upr::", "")[:60]


def load(d):
    disp = OrderedDict()
    for root, _, files in os.walk(d):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    k = int(r["Dispatch_Id"])
                    e = disp.setdefault(k, {"name": r["Kernel_Name"], "grid": r["Grid_Size"], "wg": r["Workgroup_Size"],
                                            "vgpr": r["VGPR_Count"], "agpr": r["Accum_VGPR_Count"],
                                            "lds": r["LDS_Block_Size"],
                                            "us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
                    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [disp[k] for k in sorted(disp)]


def main():
    args = sys.argv[1:]
    match, min_us = None, 20.0
    if "--match" in args:
        i = args.index("--match"); match = args[i + 1]; del args[i:i + 2]
    if "--min-us" in args:
        i = args.index("--min-us"); min_us = float(args[i + 1]); del args[i:i + 2]
    passes = [load(d) for d in args]
    n = min(len(p) for p in passes)
    # the last forward: dispatches after the last cast_f32_f16 that precedes the final one
    names = [short(e["name"]) for e in passes[0][:n]]
    ends = [i for i, s in enumerate(names) if "cast_f32_f16" in s]
    lo = ends[-2] + 1 if len(ends) >= 2 else 0
    for i in range(lo, n):
        m = {}
        for p in passes:
            m.update({k: v for k, v in p[i].items() if k not in ("us",)})
        us = passes[0][i]["us"]
        s = short(m["name"])
        if us < min_us or (match and match not in s):
            continue
        w = m.get("SQ_WAVE_CYCLES", 0) or 1
        mf = m.get("SQ_INSTS_MFMA", 0) or 1
        out = f"{us:7.1f}us {s:52s} vgpr {m['vgpr']:>3}+{m['agpr']:>3} lds {m['lds']:>6} wg {m['wg']:>4}"
        if "SQ_WAVE_CYCLES" in m:
            out += (f" | wait {m.get('SQ_WAIT_ANY', 0) / w:.2f} winst {m.get('SQ_WAIT_INST_ANY', 0) / w:.2f}"
                    f" act {m.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")
            if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                out += f" mfma_busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 256 * 4):.2f}"
        if "SQ_INSTS_MFMA" in m:
            out += (f" | /mfma valu {m.get('SQ_INSTS_VALU', 0) / mf:.1f} lds {m.get('SQ_INSTS_LDS', 0) / mf:.2f}"
                    f" salu {m.get('SQ_INSTS_SALU', 0) / mf:.1f}"
                    f" conf {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_LDS_IDX_ACTIVE', 0)):.2f}")
        if "FETCH_SIZE" in m:
            out += f" | fetch {m['FETCH_SIZE'] * 2 / 1e6:.0f}MB"
        if "WRITE_SIZE" in m:
            out += f" write {m['WRITE_SIZE'] / 1e6:.0f}MB"
        print(out)


if __name__ == "__main__":
    main()
