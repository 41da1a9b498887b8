"""Static instruction mix per device function of a gfx950 assembly listing (hipcc --offload-device-only
-S): total, VALU, scratch and global memory instructions, s_swappc calls."""
import re
import sys

for f in sys.argv[1:]:
    txt = open(f).read()
    for fn in re.split(r"\n(?=_Z[\w.]+:)", txt):
        name = fn.split(":", 1)[0].strip()
        if not name.startswith("_Z"):
            continue
        lines = [l.strip() for l in fn.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
        cnt = lambda p: sum(1 for l in lines if l.startswith(p))  # noqa: E731
        print(f"{f.split('/')[-1]:12s} {name[:60]:60s} instr {len(lines):6d} valu {cnt('v_'):6d} "
              f"scratch {cnt('scratch_'):4d} global {cnt('global_'):4d} calls {cnt('s_swappc'):3d}")
