"""Map the PCs of a crash trace (glog-style '@ 0x... ' lines, as rocprofv3's signal
handler prints them) to shared object + offset with the process's /proc/self/maps,
and name the symbol when the object is on this host (same image as the GPU box):
    python tools/exit_maps.py crash.log maps.txt
"""
import re
import subprocess
import sys


def load_maps(path):
    out = []
    for line in open(path):
        parts = line.split()
        if len(parts) < 6 or not parts[5].startswith("/"):
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        out.append((lo, hi, int(parts[2], 16), parts[5]))
    return out


def symbolize(obj, off):
    try:
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-symbolizer", "--obj=" + obj, hex(off)],
                           capture_output=True, text=True, timeout=60)
        return r.stdout.strip().splitlines()[0] if r.stdout.strip() else "?"
    except (OSError, subprocess.TimeoutExpired, IndexError):
        return "?"


def main(log, maps):
    regions = load_maps(maps)
    pcs = [int(m.group(1), 16) for m in re.finditer(r"@\s+(0x[0-9a-f]+)", open(log).read())]
    pcs += [int(m.group(1), 16) for m in re.finditer(r"PC: @\s+(0x[0-9a-f]+)", open(log).read())]
    seen = set()
    for pc in pcs:
        if pc in seen:
            continue
        seen.add(pc)
        hit = [(lo, hi, off, obj) for lo, hi, off, obj in regions if lo <= pc < hi]
        if not hit:
            print(f"{pc:#x}  (no mapping)")
            continue
        lo, hi, off, obj = hit[0]
        # file offset -> the object's virtual address: mapping offset + (pc - start);
        # for a shared object whose text segment's vaddr == its file offset this is
        # what the symbolizer takes
        foff = off + (pc - lo)
        print(f"{pc:#x}  {obj}+{foff:#x}  {symbolize(obj, foff)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
