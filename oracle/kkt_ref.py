"""Pure-Python restatement of src/utils/data_loader.rs — TEST INFRASTRUCTURE (oracle).

Follows parse_dmx (:68-156), parse_qfc (:166-198) and load_kkt_system (:211-259)
line by line, building triplets and summing duplicates like faer's
``SparseColMat::try_new_from_triplets``. Used to check the product's native
loader (tpl_load_kkt_system) on the committed fixtures.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


class LoaderError(Exception):
    pass


def _usize(s: str) -> int:
    t = s[1:] if s.startswith("+") else s
    if not t or not t.isdigit() or not t.isascii():
        raise LoaderError(f"Parse error: Failed to parse integer from '{s}'")
    return int(t)


def parse_dmx(path):
    num_nodes = num_arcs = 0
    found = False
    rows, cols, vals = [], [], []
    arc = 0
    with open(path, "r") as f:
        for line in f:
            parts = line.split()
            if not parts:
                continue
            if parts[0] == "c":
                continue
            if parts[0] == "p":
                if len(parts) >= 4 and parts[1] == "min":
                    num_nodes, num_arcs = _usize(parts[2]), _usize(parts[3])
                    found = True
                else:
                    raise LoaderError("Format error: The 'p min' problem line was not found or "
                                      "was malformed.")
            elif parts[0] == "a":
                u, v = _usize(parts[1]), _usize(parts[2])
                if u == 0:
                    raise LoaderError(f"Format error: Invalid node index '{parts[1]}'. DIMACS "
                                      "format requires 1-based positive integers.")
                if v == 0:
                    raise LoaderError(f"Format error: Invalid node index '{parts[2]}'. DIMACS "
                                      "format requires 1-based positive integers.")
                rows += [u - 1, v - 1]
                cols += [arc, arc]
                vals += [1.0, -1.0]
                arc += 1
    if not found:
        raise LoaderError("Format error: The 'p min' problem line was not found or was malformed.")
    e = sp.coo_matrix((vals, (rows, cols)), shape=(num_nodes, num_arcs)).tocsc()
    e.sum_duplicates()
    return num_nodes, num_arcs, e


def parse_qfc(path, expected_arcs):
    with open(path, "r", newline="\n") as f:
        lines = [l[:-1] if l.endswith("\n") else l for l in f]
    lines = [l[:-1] if l.endswith("\r") else l for l in lines]
    if not lines:
        raise LoaderError("Format error: Unexpected end of file while reading data.")
    m = _usize(lines[0]) if lines[0].strip() == lines[0] else None
    if m is None:
        raise LoaderError("Parse error: Failed to parse integer from 'm'")
    if m != expected_arcs:
        raise LoaderError(f"Dimension mismatch: qfc file specifies {m} arcs, but dmx file has "
                          f"{expected_arcs}.")
    out = []
    for line in lines[1 + expected_arcs: 1 + 2 * expected_arcs]:
        try:
            if line != line.strip():
                raise ValueError
            out.append(float(line))
        except ValueError:
            raise LoaderError(f"Parse error: Failed to parse float from '{line}'") from None
    return out


def load_kkt_system(dmx, qfc):
    p, m, e = parse_dmx(dmx)
    q = parse_qfc(qfc, m)
    n = p + m
    r, c, v = [], [], []
    for i, cost in enumerate(q):
        r.append(i); c.append(i); v.append(cost)
    ec = e.tocoo()
    for rr, cc, vv in zip(ec.row, ec.col, ec.data):
        r += [rr + m, cc]
        c += [cc, rr + m]
        v += [vv, vv]
    a = sp.coo_matrix((np.array(v, dtype=np.float64), (np.array(r), np.array(c))),
                      shape=(n, n)).tocsr()
    a.sum_duplicates()
    a.sort_indices()
    return a, p, m
