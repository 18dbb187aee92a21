#!/usr/bin/env python3
"""CPU emulation: would spatial splits (SBVH) shorten the bounce traversal?  Builds, in Python, a binned-SAH
hierarchy (object splits only, the product builder's rule) and the same with spatial splits (triangle
references clipped at the split plane, so a big triangle can sit in several leaves), and walks both with
path-traced bounce rays (margin_emul.py's ray generator) in nearest-first order, pruning by the best hit so
far, with the kernel's back-face cone and scalar box margin a + b R.  Prints node box tests and triangle
tests per ray for each tree (and for the product's own tree from hrt_debug_bvh_build as a check).

    python3 tools/sbvh_emul.py cave 1500 3
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import SceneCase  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "cave"
NR = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
LEAF = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ALPHA = float(os.environ.get("ALPHA", "1e-5"))
BINS = int(os.environ.get("BINS", "16"))
case = SceneCase(scene, (64, 64), 1, 1)
T = case.tris
idx = np.concatenate([np.arange(m["first_index"], m["first_index"] + m["len"]) for m in case.meshes])
A = T["a"][idx, :3].astype(np.float64)
E1 = T["edge_one"][idx, :3].astype(np.float64)
E2 = T["edge_two"][idx, :3].astype(np.float64)
NRM = T["normal"][idx, :3].astype(np.float64)
B, C = A + E1, A + E2
keep = np.linalg.norm(NRM, axis=1) > 0
nn = np.maximum(np.linalg.norm(NRM, axis=1), 1e-30)
nh = NRM / nn[:, None]
ntri = len(A)
eps, tau = 2.0 ** -24, 3e-3
rho = np.linalg.norm(NRM - np.cross(E1, E2), axis=1) / nn + 1e-12
g = np.maximum(np.linalg.norm(E1, axis=1), np.linalg.norm(E2, axis=1)) / nn
tlo = np.minimum(np.minimum(A, B), C)
thi = np.maximum(np.maximum(A, B), C)
ext = (thi - tlo).max(1)
inv_tpi = 1.02 / (tau - rho - 4e-7)
a_tri = 2.02 * ext * (6 * eps + (1.01 * rho + 3.2 * eps) * inv_tpi)
b_tri = 2.02 * ext * 18.4 * eps * g * inv_tpi
rho_max = rho.max()
inv_tp = 1.02 / (tau - rho_max - 4e-7)
abs_coef = 2.1 * (4.2 * eps + rho_max) * inv_tp
rel_t = 2.1 * (3.2 * eps + rho_max) * inv_tp + 4 * eps
print(f"{scene}: {ntri} triangles, leaf {LEAF}, bins {BINS}, alpha {ALPHA}", flush=True)


def area(lo, hi):
    e = np.maximum(hi - lo, 0.0)
    return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[0] * e[2])


def clip_bounds(t, lo, hi):
    """Bounds of triangle t clipped to the box [lo, hi] (None if empty)."""
    poly = [A[t], B[t], C[t]]
    for k in range(3):
        for side in (0, 1):
            out = []
            n = len(poly)
            for i in range(n):
                p, q = poly[i], poly[(i + 1) % n]
                if side == 0:
                    pin, qin = p[k] >= lo[k], q[k] >= lo[k]
                    plane = lo[k]
                else:
                    pin, qin = p[k] <= hi[k], q[k] <= hi[k]
                    plane = hi[k]
                if pin:
                    out.append(p)
                if pin != qin:
                    s = (plane - p[k]) / (q[k] - p[k])
                    r = p + (q - p) * s
                    r = r.copy()
                    r[k] = plane
                    out.append(r)
            poly = out
            if not poly:
                return None
    P = np.array(poly)
    return np.maximum(P.min(0), lo), np.minimum(P.max(0), hi)


class Node:
    __slots__ = ("lo", "hi", "kids", "prims", "a", "b", "axis", "cph", "sph")


def finish(node, tris):
    node.a = a_tri[tris].max()
    node.b = b_tri[tris].max()
    ax = nh[tris].sum(0)
    an = np.linalg.norm(ax)
    node.axis, node.cph, node.sph = np.array([1.0, 0, 0]), 0.0, 1.0
    if an > 1e-9:
        ax = ax / an
        phi = np.arccos(np.clip(nh[tris] @ ax, -1, 1)).max() + 1e-6
        if phi < np.pi / 2:
            node.axis, node.cph, node.sph = ax, np.cos(phi), np.sin(phi)


def subtree_tris(node):
    if node.prims is not None:
        return node.prims
    return np.unique(np.concatenate([subtree_tris(k) for k in node.kids]))


stats = {"spatial": 0, "object": 0, "refs": 0}


def build(refs, root_area, spatial, depth=0):
    """refs: list of (tri, lo, hi)."""
    node = Node()
    los = np.array([r[1] for r in refs])
    his = np.array([r[2] for r in refs])
    node.lo, node.hi = los.min(0), his.max(0)
    n = len(refs)
    node.kids, node.prims = None, None
    if n <= LEAF or depth > 60:
        node.prims = np.array(sorted({r[0] for r in refs}))
        stats["refs"] += len(node.prims)
        finish(node, node.prims)
        return node
    cent = (los + his) * 0.5
    clo, chi = cent.min(0), cent.max(0)
    best = (np.inf, None)
    for k in range(3):
        if not chi[k] > clo[k]:
            continue
        sc = BINS / (chi[k] - clo[k])
        j = np.clip(((cent[:, k] - clo[k]) * sc).astype(int), 0, BINS - 1)
        for s in range(1, BINS):
            L = j < s
            nl = int(L.sum())
            if nl == 0 or nl == n:
                continue
            c = area(los[L].min(0), his[L].max(0)) * nl + area(los[~L].min(0), his[~L].max(0)) * (n - nl)
            if c < best[0]:
                best = (c, ("obj", k, s, clo[k], sc))
    if best[1] is None:
        order = np.arange(n)
        Lm = order < n // 2
        best = (np.inf, ("mask", Lm))
    # spatial split
    sp_best = (np.inf, None)
    if spatial and best[1][0] == "obj":
        _, k, s, c0, sc = best[1]
        j = np.clip(((cent[:, k] - c0) * sc).astype(int), 0, BINS - 1)
        L = j < s
        ilo, ihi = np.maximum(los[L].min(0), los[~L].min(0)), np.minimum(his[L].max(0), his[~L].max(0))
        lam = area(ilo, ihi) if np.all(ihi > ilo) else 0.0
        if lam / root_area > ALPHA:
            for k in range(3):
                lo_k, hi_k = node.lo[k], node.hi[k]
                if not hi_k > lo_k:
                    continue
                w = (hi_k - lo_k) / BINS
                blo = [np.full(3, np.inf) for _ in range(BINS)]
                bhi = [np.full(3, -np.inf) for _ in range(BINS)]
                ent = np.zeros(BINS, int)
                ex = np.zeros(BINS, int)
                for (t, rlo, rhi) in refs:
                    b0 = min(BINS - 1, max(0, int((rlo[k] - lo_k) / w)))
                    b1 = min(BINS - 1, max(0, int((rhi[k] - lo_k) / w)))
                    ent[b0] += 1
                    ex[b1] += 1
                    for bb in range(b0, b1 + 1):
                        slo, shi = rlo.copy(), rhi.copy()
                        slo[k] = max(rlo[k], lo_k + bb * w)
                        shi[k] = min(rhi[k], lo_k + (bb + 1) * w) if bb < BINS - 1 else rhi[k]
                        cb = clip_bounds(t, slo, shi) if b0 != b1 else (slo, shi)
                        if cb is None:
                            continue
                        blo[bb] = np.minimum(blo[bb], cb[0])
                        bhi[bb] = np.maximum(bhi[bb], cb[1])
                for s in range(1, BINS):
                    nl, nr = int(ent[:s].sum()), int(ex[s:].sum())
                    if nl == 0 or nr == 0 or (nl == n and nr == n):
                        continue
                    llo = np.min(blo[:s], axis=0)
                    lhi = np.max(bhi[:s], axis=0)
                    rlo_ = np.min(blo[s:], axis=0)
                    rhi_ = np.max(bhi[s:], axis=0)
                    c = area(llo, lhi) * nl + area(rlo_, rhi_) * nr
                    if c < sp_best[0]:
                        sp_best = (c, (k, lo_k + s * w))
    if sp_best[0] < best[0]:
        k, plane = sp_best[1]
        Lr, Rr = [], []
        for (t, rlo, rhi) in refs:
            if rhi[k] <= plane:
                Lr.append((t, rlo, rhi))
            elif rlo[k] >= plane:
                Rr.append((t, rlo, rhi))
            else:
                h1 = rhi.copy()
                h1[k] = plane
                l2 = rlo.copy()
                l2[k] = plane
                c1 = clip_bounds(t, rlo, h1)
                c2 = clip_bounds(t, l2, rhi)
                if c1 is not None:
                    Lr.append((t, c1[0], c1[1]))
                if c2 is not None:
                    Rr.append((t, c2[0], c2[1]))
        if Lr and Rr and not (len(Lr) == n and len(Rr) == n):
            stats["spatial"] += 1
            node.kids = [build(Lr, root_area, spatial, depth + 1), build(Rr, root_area, spatial, depth + 1)]
            finish(node, subtree_tris(node))
            return node
    stats["object"] += 1
    if best[1][0] == "obj":
        _, k, s, c0, sc = best[1]
        j = np.clip(((cent[:, k] - c0) * sc).astype(int), 0, BINS - 1)
        Lm = j < s
    else:
        Lm = best[1][1]
    Lr = [r for r, m in zip(refs, Lm) if m]
    Rr = [r for r, m in zip(refs, Lm) if not m]
    node.kids = [build(Lr, root_area, spatial, depth + 1), build(Rr, root_area, spatial, depth + 1)]
    finish(node, subtree_tris(node))
    return node


def hit_all(o, d, tris):
    ao = o - A[tris]
    dn = NRM[tris] @ d
    det = -dn
    with np.errstate(all="ignore"):
        t = (ao * NRM[tris]).sum(1) / det
        dao = np.cross(ao, d)
        u = (E2[tris] * dao).sum(1) / det
        v = -(E1[tris] * dao).sum(1) / det
    ok = (dn < 0) & (t > 0.001) & (u >= 0) & (v >= 0) & (1 - u - v >= 0)
    if not ok.any():
        return np.inf, -1
    t = np.where(ok, t, np.inf)
    j = int(np.argmin(t))
    return t[j], int(tris[j])


ALL = np.arange(ntri)[keep]
rng = np.random.default_rng(7)
pc = case.push(1)
M = np.array(pc.cam_alignment_mat, np.float64)
cam = np.array(pc.cam_pos[:3], np.float64)
cen = np.asarray(case.rays["sample_centre"], np.float64)[:, :3]
bounce = []
tries = 0
while len(bounce) < NR and tries < 50000:
    tries += 1
    c = cen[rng.integers(len(cen))]
    w = np.array([M[0] * c[0] + M[4] * c[1] + M[8] * c[2], M[1] * c[0] + M[5] * c[1] + M[9] * c[2],
                  M[2] * c[0] + M[6] * c[1] + M[10] * c[2]])
    o, d = cam.copy(), w / np.linalg.norm(w)
    for _ in range(9):
        t, j = hit_all(o, d, ALL)
        if j < 0:
            break
        o = o + d * t
        s_ = rng.normal(size=3)
        s_ /= np.linalg.norm(s_)
        d = nh[j] + s_
        d /= np.linalg.norm(d)
        bounce.append((o.copy(), d.copy()))
bounce = bounce[:NR]
print("bounce rays", len(bounce), flush=True)


def box_enter(node, o, inv, t_lo, t_hi, R):
    f = np.maximum(o - node.lo, node.hi - o)
    Rm = min(np.sqrt(f @ f) * 1.0001, R)
    mg = node.a + node.b * Rm
    with np.errstate(invalid="ignore"):
        t0 = (node.lo - mg - o) * inv
        t1 = (node.hi + mg - o) * inv
    tn = max(t_lo, np.nanmax(np.minimum(t0, t1)))
    tf = min(t_hi, np.nanmin(np.maximum(t0, t1)))
    return tn if tn <= tf * (1 + 1e-6) + 1e-12 else None


def cone_pass(node, d):
    x = node.axis @ d
    s = np.sqrt(max(1 - x * x, 0))
    return not (x * node.cph - s * node.sph > 1e-5)


def walk(root, o, d, R):
    abs_t = abs_coef * R
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    best, bj = np.inf, -1
    boxes = prims = pops = 0
    stack = [root]
    while stack:
        node = stack.pop()
        pops += 1
        if node.prims is not None:
            prims += len(node.prims)
            t, j = hit_all(o, d, node.prims)
            if t < best:
                best, bj = t, j
            continue
        hits = []
        for k in node.kids:
            boxes += 1
            if not cone_pass(k, d):
                continue
            tn = box_enter(k, o, inv, -abs_t, (best if np.isfinite(best) else 3.4e38) * (1 + rel_t) + abs_t, R)
            if tn is not None:
                hits.append((tn, k))
        hits.sort(key=lambda x: -x[0])
        stack.extend(k for _, k in hits)
    return boxes, prims, pops, best, bj


def collapse(node, width=4):
    """The product's group collapse (make_wq_nodes): replace the inner child of largest area by its two
    children while the group has fewer than `width` members."""
    if node.prims is not None:
        return node
    ch = list(node.kids)
    while len(ch) < width:
        inner = [i for i, c in enumerate(ch) if c.prims is None]
        if not inner:
            break
        i = max(inner, key=lambda i: area(ch[i].lo, ch[i].hi))
        c = ch[i]
        ch[i:i + 1] = c.kids
    new = Node()
    for s in Node.__slots__:
        setattr(new, s, getattr(node, s))
    new.kids = [collapse(c, width) for c in ch]
    return new


def count(node):
    if node.prims is not None:
        return 1, len(node.prims)
    n, p = 1, 0
    for k in node.kids:
        a, b = count(k)
        n += a
        p += b
    return n, p


refs = [(int(t), tlo[t], thi[t]) for t in ALL]
sbox_root = area(tlo[ALL].min(0), thi[ALL].max(0))
lo_s, hi_s = tlo[ALL].min(0), thi[ALL].max(0)
trees = {}
for name, sp in (("object", False), ("spatial", True)):
    stats.update(spatial=0, object=0, refs=0)
    root = build(refs, sbox_root, sp)
    nodes, nref = count(root)
    print(f"{name}: nodes {nodes}, leaf refs {nref} ({nref / len(ALL):.2f}x), spatial splits {stats['spatial']}",
          flush=True)
    trees[name] = root
    trees[name + "4"] = collapse(root)
res = {k: np.zeros(3) for k in trees}
mism = 0
for (o, d) in bounce:
    f = np.maximum(np.abs(o - lo_s), np.abs(hi_s - o))
    R = np.sqrt(f @ f) * 1.0001
    ref = None
    for k, root in trees.items():
        b, p, q, t, j = walk(root, o, d, R)
        res[k] += (b, p, q)
        if ref is None:
            ref = j
        elif j != ref:
            mism += 1
print(f"rays {len(bounce)}, hit mismatches between trees {mism}")
for k, v in res.items():
    v = v / len(bounce)
    print(f"  {k:9s} box tests/ray {v[0]:6.1f}   triangle tests/ray {v[1]:6.1f}   pops/ray {v[2]:6.1f}")
