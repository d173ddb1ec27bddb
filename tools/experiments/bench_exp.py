"""bench.py against the experiments library (rl-quic-raptor_amd/build_exp/librqhip.so), so RQHIP_* knobs apply."""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402

rqhip.LIB_PATH = ROOT / "rl-quic-raptor_amd" / "build_exp" / "librqhip.so"
sys.argv = [str(ROOT / "bench.py")] + sys.argv[1:]
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
