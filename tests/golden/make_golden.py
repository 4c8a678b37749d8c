"""Regenerate the golden fixtures in this directory from the oracle (run from the repo root:
`python tests/golden/make_golden.py`).  The reference ships no golden vectors or fixed seeds
(SURVEY.md §4), so these fixtures are the oracle's outputs on seeded inputs; the oracle itself is
pinned by the reference's known-answer tests (oracle/test_kat.cpp).  They freeze the oracle and give
the GPU parity tests byte-exact targets that do not need the oracle at run time."""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))

import oracle_ref as orc  # noqa: E402
from gen import random_orset_pair, random_pnc  # noqa: E402


def main():
    rng = np.random.default_rng(0x6A616E7573)
    # PN-Counter, reference width (int32): 256 keys x 8 replicas, 1024 received rows with repeats,
    # a few rows crafted to overflow the checked Sum.
    AP = random_pnc(rng, 256, 8, 4, absent=False, lo=0, hi=1 << 24)
    AN = random_pnc(rng, 256, 8, 4, absent=False, lo=0, hi=1 << 24)
    BP = random_pnc(rng, 1024, 8, 4, lo=-(1 << 20), hi=1 << 25)
    BN = random_pnc(rng, 1024, 8, 4, lo=-(1 << 20), hi=1 << 25)
    keys = rng.integers(0, 256, 1024).astype(np.uint32)
    BP[:4] = np.iinfo(np.int32).max  # keys[0..3] overflow ΣP
    outP, outN = orc.pnc_merge(AP, AN, BP, BN, keys)
    values, ovf = orc.pnc_values(outP, outN)
    np.savez_compressed(HERE / "pnc_merge_i32.npz", AP=AP, AN=AN, BP=BP, BN=BN, keys=keys, outP=outP, outN=outN,
                        values=values, ovf=ovf)

    La, Lr, Ra, Rr = random_orset_pair(rng, n_sets=24, n_elems=10, pool=16)
    out_add, out_rem = orc.orset_merge(La, Lr, Ra, Rr)
    q_set = np.repeat(np.arange(25, dtype=np.uint32), 12)
    q_elem = np.tile(np.array(list(range(11)) + [orc.NULL_ELEM], np.uint32), 25)
    contains = orc.orset_contains(out_add, out_rem, q_set, q_elem)
    np.savez_compressed(HERE / "orset_merge.npz", La=La, Lr=Lr, Ra=Ra, Rr=Rr, out_add=out_add, out_rem=out_rem,
                        q_set=q_set, q_elem=q_elem, contains=contains)
    print("pnc", outP.shape, int(ovf.sum()), "orset", out_add.size, out_rem.size, int(contains.sum()))


if __name__ == "__main__":
    main()
