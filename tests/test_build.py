"""The tree builds from a clean checkout: every source of librqhip.so compiles for gfx950 and links
(into a scratch build directory, so the in-tree library the other tests load is left alone), and
the linked library exports the whole C-ABI."""
import ctypes
import re
import shutil
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "rl-quic-raptor_amd"


def test_clean_build_links(tmp_path):
    # copy the package sources (not its build/) and build them from nothing
    dst = tmp_path / "pkg"
    shutil.copytree(PKG / "csrc", dst / "csrc")
    shutil.copytree(PKG / "fecquic", dst / "fecquic")
    shutil.copy(PKG / "Makefile", dst / "Makefile")
    (tmp_path / "include").mkdir()
    for h in ("rqhip.h", "rqhip_debug.h"):
        shutil.copy(ROOT / "include" / h, tmp_path / "include" / h)
    r = subprocess.run(["make", "-s", "-C", str(dst), "-j8", "all"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    so = dst / "build" / "librqhip.so"
    for f in ("librqhip.so", "librqcpu.so", "libfecquic.so", "fecquic", "raptorq_eval"):
        assert (dst / "build" / f).exists(), f
    L = ctypes.CDLL(str(so))
    txt = re.sub(r"/\*.*?\*/", "", (ROOT / "include/rqhip.h").read_text() + (ROOT / "include/rqhip_debug.h").read_text(),
                 flags=re.S)
    for name in sorted(set(re.findall(r"\b(rq_[a-z_]+)\s*\(", txt))):
        assert hasattr(L, name), name
