"""Regenerate the netgen KKT fixtures under tests/golden/kkt (test infrastructure).

The .dmx files are the output of the reference's own NETGEN generator
(/root/reference/data/netgen/src/*.c, compiled from those sources by `make -C oracle
ref` into oracle/_ref/netgen — never the reference's prebuilt binary) run on the
recorded parameter lines below (seed line + parameter line). Each
file is xz-compressed; its decompressed md5 is pinned in tests/conftest.py (KKT_MD5)
and checked by tests/test_boundary.py.

    python tests/golden/make_fixtures.py [--check] [ARCS ...]

--check regenerates into memory and only compares md5s (what the CPU test runs).
The 5M-arc instance of BASELINE configs[4] is not a netgen fixture: it comes from the
engine's own generator (tpl_generate_kkt, seed 42).
"""
import argparse
import hashlib
import lzma
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
NETGEN = os.path.join(ROOT, "oracle", "_ref", "netgen")

# arcs -> (seed, netgen parameter line); recorded from the reference's data/ instances
PARAMS = {
    5000: ("1499034469", "1 115 6 7 5000 1 81 395 0 0 0 100 22 110"),
    50000: ("24569811", "1 365 14 9 50000 1 46 644 0 0 0 100 46 142"),
    500000: ("1545440015", "1 1155 91 7 500000 1 99 376 0 0 0 100 19 103"),
}


def generate(arcs: int) -> bytes:
    if not os.path.exists(NETGEN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True,
                       capture_output=True)
    if not os.path.exists(NETGEN):
        raise RuntimeError("oracle/_ref/netgen is not built (needs /root/reference sources)")
    seed, par = PARAMS[arcs]
    return subprocess.run([NETGEN], input=f"{seed}\n{par}\n".encode(), capture_output=True,
                          check=True).stdout


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("arcs", nargs="*", type=int, default=sorted(PARAMS))
    args = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import KKT_MD5
    bad = 0
    for arcs in args.arcs:
        out = generate(arcs)
        md5 = hashlib.md5(out).hexdigest()
        ok = md5 == KKT_MD5[arcs]
        bad += not ok
        print(f"{arcs}: {len(out)} B md5 {md5} {'ok' if ok else 'MISMATCH'}")
        if not args.check:
            with lzma.open(os.path.join(HERE, "kkt", f"netgen-{arcs}-3.dmx.xz"), "wb",
                           preset=9 | lzma.PRESET_EXTREME) as f:
                f.write(out)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
