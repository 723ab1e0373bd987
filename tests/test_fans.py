"""PMMG_precompute_nodeTrias (src/locate_pmmg.c:134-195) by rotation through
the tria adjacency, the rule of k_fan_rotate (parmmg_amd/csrc/pmx_bdy.hip),
restated on the CPU: every (tria, corner) slot turns around its vertex
through Mmg's adjt (edge i opposite vertex i) and puts its tria at its rank
in the window of the fan's smallest tria.  The lists equal the reference's
construction (each vertex's trias in increasing index order); a surface with
an edge without its neighbour, or a vertex whose fan does not hold all its
trias (a pinched vertex), is refused."""
import numpy as np

from parmmg_amd import mesh as M

FAN_CAP = 32


def pinched_cubes(n=3):
    """Two Kuhn cubes touching at one vertex, (1, 1, 1): every edge of the
    surface is manifold, the shared vertex has two separate fans."""
    a = M.kuhn_cube(n, jitter=0.0)
    xyz = np.vstack([a.xyz, a.xyz[1:] + 1.0])
    ia = int(np.nonzero(np.all(np.abs(a.xyz[1:] - 1.0) < 1e-12, axis=1))[0][0]) + 1
    ib = int(np.nonzero(np.all(np.abs(a.xyz[1:]) < 1e-12, axis=1))[0][0]) + 1
    tb = a.tet[1:] + a.np
    tb[tb == ib + a.np] = ia
    tet = np.vstack([a.tet, tb]).astype(np.int32)
    keep = np.ones(len(xyz), bool)
    keep[ib + a.np] = False
    newid = np.cumsum(keep) - 1
    tet = newid[tet].astype(np.int32)
    tet[0] = 0
    return M.from_tets(xyz[keep], tet), ia


def fans_by_rotation(tria, adjt):
    nt = len(tria) - 1
    count = {}
    for k in range(1, nt + 1):                  # the upload's check: trias per vertex
        for v in tria[k]:
            count[int(v)] = count.get(int(v), 0) + 1
    rng = {}
    lists = {}
    for k in range(1, nt + 1):
        for l in range(3):
            v = int(tria[k][l])
            cur, cx, w = k, (l + 1) % 3, int(tria[k][(l + 2) % 3])
            members = [(k, l)]
            while True:
                nxt = int(adjt[3 * (cur - 1) + 1 + cx]) // 3
                if nxt == k:
                    break
                if nxt <= 0 or len(members) == FAN_CAP:
                    return None
                tn = [int(x) for x in tria[nxt]]
                if v not in tn or w not in tn:
                    return None
                cv, cw = tn.index(v), tn.index(w)
                members.append((nxt, cv))
                cur, cx, w = nxt, cw, tn[3 - cv - cw]
            if len(members) != count[v]:        # a fan of one sheet of a pinched vertex
                return None
            own, lown = min(members)
            rank = sum(1 for g, _ in members if g < k)
            base = (3 * own + lown - 3) * FAN_CAP
            rng[(k, l)] = (base, base + len(members))
            lists[base + rank] = k
    return rng, lists


def test_rotation_fans_equal_sorted_fans():
    m = M.kuhn_cube(5)
    out = fans_by_rotation(m.tria, m.adjt)
    assert out is not None
    rng, lists = out
    nt = len(m.tria) - 1
    by_vertex = {}
    for k in range(1, nt + 1):                 # the reference's construction
        for l in range(3):
            by_vertex.setdefault(int(m.tria[k][l]), []).append(k)
    for k in range(1, nt + 1):
        for l in range(3):
            lo, hi = rng[(k, l)]
            fan = [lists[i] for i in range(lo, hi)]
            assert fan == by_vertex[int(m.tria[k][l])]


def test_open_surface_refused():
    m = M.kuhn_cube(3)
    adjt = m.adjt.copy()
    a = int(adjt[3 * (7 - 1) + 1])
    adjt[3 * (7 - 1) + 1] = 0
    adjt[3 * (a // 3 - 1) + 1 + a % 3] = 0
    assert fans_by_rotation(m.tria, adjt) is None


def test_pinched_vertex_refused():
    """Two surface sheets touching at a vertex: each fan walked around one
    sheet closes short of the vertex's tria count -- the upload keeps the
    sort (a ParMmg group pinched at a vertex by its partition)."""
    m, _ = pinched_cubes()
    assert fans_by_rotation(m.tria, m.adjt) is None
