"""Background numberings of the bench (lexicographic,
--shuffle-tets, Mmg-appended) and the walk record's escape rule
(parmmg_amd/csrc/pmx_wrec.h): CPU checks of the host helpers."""
import numpy as np
import pytest

from parmmg_amd import mesh as M


def faces_match(m):
    """Every adjacency entry joins two tets sharing the 3 face vertices."""
    t = m.tet
    ad = m.adja[1:4 * m.ne + 1].reshape(m.ne, 4)
    k, f = np.nonzero(ad > 0)
    k1 = k + 1
    kn, fn = ad[k, f] >> 2, ad[k, f] & 3
    for a, fa, b, fb in zip(k1[:2000], f[:2000], kn[:2000], fn[:2000]):
        fa_v = sorted(np.delete(t[a], fa))
        fb_v = sorted(np.delete(t[b], fb))
        if fa_v != fb_v:
            return False
        if (m.adja[4 * (b - 1) + 1 + fb] >> 2) != a:
            return False
    return True


@pytest.mark.parametrize("kind", ["lex", "shuffle", "appended"])
def test_numbering_keeps_the_mesh(kind):
    m = M.kuhn_cube(6)
    mm, tinv = M.numbering(m, kind)
    assert mm.ne == m.ne and mm.np == m.np
    assert faces_match(mm)
    if tinv is not None:
        assert np.array_equal(mm.tet[tinv[1:]], m.tet[1:])      # same tets, moved
        assert sorted(tinv[1:].tolist()) == list(range(1, m.ne + 1))
    if kind == "appended":                                      # 10 % at the end, order kept
        moved = tinv[1:] > m.ne - m.ne // 10
        assert moved.sum() == m.ne // 10
        assert np.all(np.diff(tinv[1:][~moved]) > 0) and np.all(np.diff(tinv[1:][moved]) > 0)


def test_wrec_escape_rule():
    """The escape rule of the 24-B walk records: deltas within the fields
    encode, one past the limits escapes (vertex: 20-bit, neighbour: 24-bit
    with -2^23 reserved for boundary faces)."""
    m = M.kuhn_cube(3)
    assert M.wrec_escapes(m) == 0
    big = m.tet.copy()
    big[5, 3] = big[5, 0] + (1 << 19)
    mm = M.Mesh(m.xyz, big, m.adja, m.tria, m.adjt)
    assert M.wrec_escapes(mm) == 1
    big[5, 3] = big[5, 0] + (1 << 19) - 1
    assert M.wrec_escapes(M.Mesh(m.xyz, big, m.adja, m.tria, m.adjt)) == 0


def test_wrec_far_field_rule():
    """A neighbour delta past the 24-bit field escapes that field only
    (-2^23 is the boundary code, -2^23 + 1 the far code); an appended
    numbering of more than 2^23 tets puts its moved tets' faces there."""
    m = M.kuhn_cube(3)
    assert M.wrec_far_fields(m) == (0, 0)
    ad = m.adja.copy()
    # tet 1's face 0 neighbour moved by > 2^23 (out of range on purpose:
    # the rule is about the delta, not the mesh)
    k, f = 1, int(np.nonzero(ad[1:5] > 0)[0][0])
    for d, far in (((1 << 23) - 1, 0), (1 << 23, 1)):
        ad[4 * (k - 1) + 1 + f] = (k + d) * 4
        assert M.wrec_far_fields(M.Mesh(m.xyz, m.tet, ad, m.tria, m.adjt))[0] == far
    assert M.wrec_escapes(M.Mesh(m.xyz, m.tet, ad, m.tria, m.adjt)) == 0
