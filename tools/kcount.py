"""Per-kernel instruction histogram and register counts from a hipcc --save-temps .s file.

    python tools/kcount.py build/factor-hip-amdgcn-amd-amdhsa-gfx950.s tiles_x3
"""
import collections
import re
import sys


def main(path, pat):
    s = open(path).read()
    meta = s[s.find("amdhsa.kernels"):]
    for m in re.finditer(r"^(_Z\w*%s\w*):" % pat, s, re.M):
        name, start = m.group(1), m.end()
        body = s[start:s.find(".Lfunc_end", start)]
        c = collections.Counter()
        for line in body.splitlines():
            line = line.split(";")[0].strip()
            if line and not line.startswith((".", "/")) and not line.endswith(":"):
                c[line.split()[0]] += 1
        print(name, sum(c.values()))
        print("  ", ", ".join("%s %d" % kv for kv in c.most_common(18)))
        i = meta.find(".name:           " + name)
        j = meta.find("\n  - ", i) if i >= 0 else -1
        blk = meta[meta.rfind("\n  - ", 0, i):j if j > 0 else len(meta)] if i >= 0 else ""
        print("  ", re.findall(r"\.(vgpr_count|agpr_count|sgpr_count|vgpr_spill_count|group_segment_fixed_size):\s+(\d+)", blk))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
