"""Per-object round trips (K=5, L=1100, N=8, 10 % loss, 50 trials) through the Python mirror, and
the encoder's repairs against the oracle: a GPU regression probe for column-program launch changes.
usage: [RQHIP_LIB=...] python tools/experiments/perobj_check.py"""
import os
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "rl-quic-raptor_amd"))
sys.path.insert(0, str(ROOT))
import rqhip  # noqa: E402
from oracle import oracle as O  # noqa: E402

if os.environ.get("RQHIP_LIB"):
    rqhip.LIB_PATH = Path(os.environ["RQHIP_LIB"])

rng = random.Random(1337)
K, L, N = 5, 1100, 8
bad_rep = bad_dec = ok = 0
for t in range(50):
    data = bytes(rng.getrandbits(8) for _ in range(K * L - (t % 7) * 13))
    enc = rqhip.NewRaptorQEncoder(data, K, L)
    ref = O.OracleEncoder(data, L)
    for i in range(N):
        if bytes(enc.GenSymbol(i)) != bytes(ref.gen_symbol(i)):
            bad_rep += 1
    pk = rqhip.RaptorQEncodeBlock(data, N, K, L)
    recv = [p for p in pk if rng.random() >= 0.1]
    got, okf = rqhip.RaptorQDecodeBytes(recv, N, K, L, len(data))
    if okf:
        ok += 1
        bad_dec += bytes(got) != data
print("trials 50 ok %d bad_repair_symbols %d bad_decodes %d" % (ok, bad_rep, bad_dec))
