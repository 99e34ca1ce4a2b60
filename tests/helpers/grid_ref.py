"""numpy restatement of the host GridNeighbors CSR (usac_host.hpp; the reference's
NearestNeighbors::getGridNearestNeighbors, nearest_neighbors.cpp:160-202): cells
((int)(x1/cs), (int)(y1/cs), (int)(x2/cs), (int)(y2/cs)) by fp32 division and truncation,
numbered in order of first appearance, members ascending; eligible = points with >= m
neighbours (NAPSAC).  Test infrastructure."""
import numpy as np


def grid_csr(pts, cs, m):
    c = (np.ascontiguousarray(pts, dtype=np.float32) / np.float32(cs)).astype(np.int32)  # fp32 div, trunc
    _, first, inv = np.unique(c, axis=0, return_index=True, return_inverse=True)
    inv = inv.reshape(-1)
    new_of_old = np.empty(len(first), dtype=np.int64)
    new_of_old[np.argsort(first, kind="stable")] = np.arange(len(first))
    cell = new_of_old[inv]
    members = np.argsort(cell, kind="stable").astype(np.int32)
    size = np.bincount(cell, minlength=len(first))
    start = np.concatenate([[0], np.cumsum(size)]).astype(np.uint32)
    rank = np.empty(len(pts), dtype=np.uint32)
    rank[members] = np.arange(len(pts)) - start[cell[members]]
    eligible = np.where(size[cell] - 1 >= m)[0].astype(np.int32)
    return {"cell": cell.astype(np.uint32), "rank": rank, "start": start, "members": members, "eligible": eligible}
