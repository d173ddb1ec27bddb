"""bench.py against the experiments library (rl-quic-raptor_amd/build_exp/librqhip.so), so RQHIP_* knobs apply."""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
import rqhip  # noqa: E402

rqhip.LIB_PATH = ROOT / "rl-quic-raptor_amd" / "build_exp" / "librqhip.so"
args = sys.argv[1:]
if "--apply-lds" in args:  # RQHIP_APPLY_LDS for this process (rocprofv3 runs the program directly)
    import os
    i = args.index("--apply-lds")
    os.environ["RQHIP_APPLY_LDS"] = args[i + 1]
    del args[i:i + 2]
sys.argv = [str(ROOT / "bench.py")] + args
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
