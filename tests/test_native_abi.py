"""CPU: libkfac_hip.so loads, exports every symbol include/kfac_hip.h declares, and the
ctypes structs mirror the C structs byte for byte (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "kfac_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"KFAC_API\s+[\w\s\*]+?\b(kfac_\w+)\s*\(", src)))


def test_library_loads_and_exports_header_symbols():
    from bnn_kfac_amd import _native as N
    lib = N.lib()
    syms = declared_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in kfac_hip.h but not exported"
        assert s in N.SIGNATURES, f"{s} not bound in _native.SIGNATURES"
    assert lib.kfac_version().decode().startswith("bnn_kfac_amd")
    assert lib.kfac_strerror(-3).decode() == "workspace too small"


def test_gfx950_code_object_present():
    data = open(os.path.join(ROOT, "bnn_kfac_amd", "libkfac_hip.so"), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # the offload bundle id of the device code


@pytest.mark.parametrize("name", ["kfac_operand", "kfac_factor_job", "kfac_invert_job",
                                  "kfac_eig_job", "kfac_quad_job", "kfac_tri_job"])
def test_struct_layout_matches_header(tmp_path, name):
    from bnn_kfac_amd import _native as N
    pyname = {"kfac_operand": "Operand", "kfac_factor_job": "FactorJob",
              "kfac_invert_job": "InvertJob", "kfac_eig_job": "EigJob",
              "kfac_quad_job": "QuadJob", "kfac_tri_job": "TriJob"}[name]
    c = tmp_path / "sz.c"
    c.write_text(f'#include <stdio.h>\n#include "{HEADER}"\n'
                 f'int main(void){{printf("%zu", sizeof({name})); return 0;}}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-o", str(exe), str(c)], check=True)
    size = int(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    assert size == ctypes.sizeof(getattr(N, pyname))


def test_workspace_queries_need_no_gpu():
    from bnn_kfac_amd import _native as N
    lib = N.lib()
    op = N.Operand()
    op.ptr, op.layout, op.rows, op.cols, op.ld, op.has_ones = 1, N.ROWMAJOR, 4096, 784, 784, 1
    job = N.FactorJob()
    job.x, job.F, job.ldF = op, 1, 785
    arr = N.as_array(N.FactorJob, [job])
    ws = lib.kfac_factor_workspace_bytes(arr, 1)
    assert ws >= 91 * 64 * 64 * 4  # at least one slab per lower tile
    inv = N.InvertJob()
    inv.F, inv.ldF, inv.n, inv.out, inv.ldo = 1, 785, 785, 1, 785
    # three padded fp64 matrices (32-tiles for n <= 1536: 785 -> 800)
    assert lib.kfac_invert_workspace_bytes(N.as_array(N.InvertJob, [inv]), 1) >= 3 * 800 * 800 * 8
    # argument validation happens before any launch
    bad = N.FactorJob()
    assert lib.kfac_factor_update(N.as_array(N.FactorJob, [bad]), 1, None, 0, None) == N.KFAC_EINVAL


def test_sample_struct_layout(tmp_path):
    from bnn_kfac_amd import _native as N
    c = tmp_path / "sz.c"
    c.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "{HEADER}"\n'
                 'int main(void){printf("%zu %zu %zu", sizeof(kfac_sample_job), '
                 'offsetof(kfac_sample_job, W), offsetof(kfac_sample_job, wcols)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-o", str(exe), str(c)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == [ctypes.sizeof(N.SampleJob), N.SampleJob.W.offset, N.SampleJob.wcols.offset]
    # argument validation happens before any launch
    assert N.lib().kfac_sample(N.as_array(N.SampleJob, [N.SampleJob()]), 1, 0, None, 0,
                               None) == N.KFAC_EWORKSPACE


def test_knobs_read_once_and_settable_per_call():
    """The environment knobs are read once, at load (knobs.h): get_knob reports them,
    set_knob changes only the per-call ones; the kernel-selection ones refuse."""
    import subprocess
    import sys
    from bnn_kfac_amd import _native as N
    assert N.get_knob("KFAC_INV_GRAPH") in (0, 1)
    before = N.get_knob("KFAC_INV_LOOKAHEAD")
    N.set_knob("KFAC_INV_LOOKAHEAD", 0)
    assert N.get_knob("KFAC_INV_LOOKAHEAD") == 0
    N.set_knob("KFAC_INV_LOOKAHEAD", before)
    for name in ("KFAC_SYRK3", "KFAC_TILES_X3", "KFAC_CONV_K", "KFAC_NO_SUCH_KNOB"):
        with pytest.raises(N.NativeError):
            N.set_knob(name, 1)
    with pytest.raises(N.NativeError):
        N.get_knob("KFAC_INV_PRIO")  # an A/B knob of earlier rounds, gone
    # a fresh process sees its environment at load
    code = ("from bnn_kfac_amd import _native as N; "
            "print(N.get_knob('KFAC_SYRK3'), N.get_knob('KFAC_EIG_RB'), N.get_knob('KFAC_CONV_K'))")
    env = dict(os.environ, KFAC_SYRK3="1", KFAC_EIG_RB="8", KFAC_CONV_K="3")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True,
                         env=env, cwd=ROOT).stdout.split()
    assert out == ["1", "8", "3"]
