"""Per-kernel register / scratch / LDS usage from a hipcc --cuda-device-only -S output (.s).
python tools/kmeta.py file.s [name-filter]"""
import re
import sys

text = open(sys.argv[1]).read()
meta = text[text.find("amdhsa.kernels:"):]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"\.(\w+):\s+(\S+)", blk))
    name = f.get("name", "?")
    if flt in name:
        print(f"vgpr {f.get('vgpr_count','?'):>4} agpr {f.get('agpr_count','?'):>4} sgpr {f.get('sgpr_count','?'):>4} "
              f"spill v{f.get('vgpr_spill_count','?')}/s{f.get('sgpr_spill_count','?')} "
              f"scratch {f.get('private_segment_fixed_size','?'):>4} lds {f.get('group_segment_fixed_size','?'):>6}  {name[:90]}")
