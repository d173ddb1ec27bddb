"""CPU-only worker for spawned oracle pools in GPU tests: imports numpy and the oracle, nothing that
touches a GPU (no torch, no librqhip)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent


def oracle_repairs(args):
    """The oracle's repair symbols (rows esis) of one block: (data bytes, T, esis) -> [len(esis), T]."""
    data, T, esis = args
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    from oracle import oracle as O
    enc = O.OracleEncoder(data, T)
    return np.stack([enc.gen_symbol(e) for e in esis])


def oracle_decode(args):
    """The oracle decoder on one block: (K, T, {esi: row bytes} of the received symbols) -> (ok, payload)."""
    K, T, recv = args
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    from oracle import oracle as O
    dec = O.OracleDecoder(K * T, T)
    for esi, row in recv.items():
        dec.add_symbol(esi, row)
    return dec.decode()
