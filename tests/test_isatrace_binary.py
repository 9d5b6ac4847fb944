"""Precompiled code objects -> reassemblable assembly (isatrace/binary.py):
every function and kernel descriptor of the suite's gfx950 code objects
comes back byte-identical from its own listing.  Host-only (llvm tools)."""
import glob
import os
import shutil
import subprocess

import pytest

from accel_sim_framework_distributed_amd.isatrace import binary as B

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
APPS = sorted(glob.glob(os.path.join(REPO, "bin", "apps", "*")))

pytestmark = pytest.mark.skipif(not APPS or not os.path.exists(os.path.join(B.LLVM, "llvm-objdump")),
                                reason="needs the built apps and the ROCm llvm tools")


@pytest.mark.parametrize("app", ["nw", "lud", "heartwall", "power_suite"])
def test_roundtrip_byte_identical(app, tmp_path):
    exe = os.path.join(REPO, "bin", "apps", app)
    if not os.path.exists(exe):
        pytest.skip(f"{app} not built")
    cos = B.extract(exe, str(tmp_path / "x"))
    assert len(cos) == 1
    r = B.roundtrip(cos[0], str(tmp_path / "rt"))
    assert r["functions"] >= 1 and r["identical"] == r["functions"], r["mismatch"]
    assert r["kd_identical"] and r["data_identical"]
    assert r["unsupported"] == []


def test_roundtrip_calls_and_globals(tmp_path):
    """Direct calls to device functions and addresses of __constant__ /
    __device__ variables (s_getpc_b64 + literal pairs) become relocations and
    resolve to the same symbols after reassembly."""
    co = str(tmp_path / "calls.co")
    src = os.path.join(REPO, "tests", "data", "binary_calls.hip")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-c", src, "-o", co],
                   check=True, capture_output=True)
    cos = B.extract(co, str(tmp_path / "x"))
    assert len(cos) == 1
    r = B.roundtrip(cos[0], str(tmp_path / "rt"))
    assert r["functions"] == 3 and r["identical"] == 3 and r["pcrel"] == 4, r
    assert r["kd_identical"] and r["data_identical"] and r["unsupported"] == []


def test_listing_is_instrumentable(tmp_path):
    """The recovered listing goes through the same rewriter as compiler
    output (segment / memory probes) and assembles."""
    from accel_sim_framework_distributed_amd.isatrace import rewrite
    cos = B.extract(os.path.join(REPO, "bin", "apps", "nw"), str(tmp_path / "x"))
    lst = B.disassemble(cos[0])
    new, maps = rewrite.instrument(lst.asm())
    assert {m.name for m in maps} == {f.name for f in lst.funcs if f.kernel}
    B.assemble(new, str(tmp_path / "instr.co"))


def test_unsupported_constructs_are_named():
    f = B.Func("k", 0, 32, True, [("s_getpc_b64 s[0:1]", 0, b""), ("s_mov_b32 s2, 0", 4, b""),
                                  ("s_setpc_b64 s[4:5]", 8, b"")])
    B._resolve_pcrel(f)
    bad = B.unsupported(B.Listing("x", [f], {}, "", 4))
    assert any("s_getpc_b64 not followed" in b for b in bad) and any("indirect branch" in b for b in bad)
