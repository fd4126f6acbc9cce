"""Per-kernel ISA statistics from a hipcc -save-temps .s file: registers,
occupancy, and instruction counts of the hottest loop (the largest basic
block between a label and its backward branch).

Usage: python tools/isa_stats.py <file.s> <symbol-substring>..."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for m in re.finditer(r"^(_Z\S*" + re.escape(pat) + r"\S*):[^\n]*\n", s, re.M):
        name = m.group(1)
        i = m.end()
        j = s.find(".Lfunc_end", i)
        meta = s[j:j + 4000]
        g = lambda k: (re.search(r"; " + k + r": (\d+)", meta) or [None, "?"])[1]
        body = s[i:j]
        # loops: label ... s_cbranch back to it
        lines = body.split("\n")
        labels = {m.group(1): n for n, l in enumerate(lines) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
        best, bestkey = None, None
        for n, l in enumerate(lines):
            mm = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)", l) or re.match(r"\s+s_branch\s+(\.LBB\S+)", l)
            if mm and mm.group(1) in labels and labels[mm.group(1)] < n:
                seg = lines[labels[mm.group(1)]:n + 1]
                ins = [x.split()[0] for x in seg if x.startswith("\t") and not x.strip().startswith((".", ";"))]
                key = (sum(x.startswith(("v_fma_f64", "v_fmac_f64", "v_fma_f32", "v_fmac_f32", "v_mfma")) for x in ins), len(ins))
                if best is None or key > bestkey:
                    best, bestkey = ins, key
        c = Counter(best or [])
        v = sum(k.startswith("v_") for k in best or [])
        print(f"{name[:70]}\n  vgpr {g('NumVgprs')} agpr {g('NumAgprs')} sgpr {g('NumSgprs')} scratch {g('ScratchSize')}"
              f" occupancy {g('Occupancy')} lds {g('LDSByteSize') if 'LDSByteSize' in meta else '?'}")
        if best:
            print(f"  hottest loop: {len(best)} instr, VALU {v}, fma64 {c['v_fma_f64'] + c['v_fmac_f64_e32']}, "
                  f"ds_read {sum(n for k, n in c.items() if k.startswith('ds_read'))}, "
                  f"s_load {sum(n for k, n in c.items() if k.startswith('s_load'))}, "
                  f"s_waitcnt {c['s_waitcnt']}, SALU {sum(n for k, n in c.items() if k.startswith('s_') and not k.startswith(('s_load', 's_waitcnt', 's_cbranch', 's_branch')))}")
