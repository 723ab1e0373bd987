"""Background topology on the GPU: tet face adjacency
(MMG3D_hashTetra), boundary trias (MMG5_chkBdryTria) and their edge adjacency
(MMG3D_hashTria), against the CPU builders of parmmg_amd/csrc/meshgen.c.

The adjacency of a valid mesh is unique, so it is compared exactly; boundary
trias are compared in the (tet, face) order both builders use.  Mmg itself is
absent: its own tria order is not verified (parity unpinned for that order).
"""
import os

import numpy as np
import pytest

from conftest import REF_INPUTS
from parmmg_amd import mesh as M

pytestmark = pytest.mark.gpu


def shuffled(m, seed=7):
    """Same mesh, tets in a random order and local vertices rotated (keeps
    the orientation): a non-lattice numbering."""
    rng = np.random.default_rng(seed)
    perm = rng.permutation(m.ne) + 1
    tet = np.zeros_like(m.tet)
    tet[1:] = m.tet[perm]
    even = [[0, 1, 2, 3], [1, 0, 3, 2], [2, 3, 0, 1], [3, 2, 1, 0]]
    rot = rng.integers(0, 4, m.ne)
    tet[1:] = np.take_along_axis(tet[1:], np.array(even)[rot], axis=1)
    return M.from_tets(m.xyz, tet)


@pytest.mark.parametrize("case", ["kuhn6", "kuhn17", "shuffled", "wave"])
def test_adjacency_and_boundary(transfer, case):
    if case == "kuhn6":
        m = M.kuhn_cube(6)
    elif case == "kuhn17":
        m = M.kuhn_cube(17)
    elif case == "shuffled":
        m = shuffled(M.kuhn_cube(9))
    else:
        m = M.read_medit(os.path.join(REF_INPUTS, "wave.0.mesh"))
    adja = transfer.build_adja(m.tet, m.np)
    assert np.array_equal(adja, m.adja)
    tria, adjt = transfer.build_bdry(m.tet, m.np, adja)
    assert np.array_equal(tria, m.tria)
    assert np.array_equal(adjt, m.adjt)


def test_upload_without_adjacency(transfer):
    """pmx_upload_background with adja == NULL builds it on the device: the
    transfer gives the same result as with the host adjacency."""
    from parmmg_amd.transfer import mesh_view  # noqa: F401
    m = M.kuhn_cube(7)
    x, t = M.new_points(7, surface=False)
    sols = [M.on_vertices(m, M.iso_metric)]
    transfer.upload_background(m, sols, 0)
    transfer.upload_points(x, t)
    transfer.run()
    a = transfer.download()
    m2 = M.Mesh(m.xyz, m.tet, None, m.tria, m.adjt, m.hausd)
    transfer.upload_background(m2, sols, 0)
    transfer.upload_points(x, t)
    transfer.run()
    b = transfer.download()
    assert np.array_equal(a.elem, b.elem)
    assert np.array_equal(a.sols[0].view(np.int64), b.sols[0].view(np.int64))


def test_upload_device_adjacency_chunked_and_refused(transfer):
    """The device face matching runs on the topology stream beside the
    solutions' upload: at a size where the connectivity goes down in several
    chunks (ne > 2^21) the located elements and fields equal those of the
    host-adjacency upload bit for bit; a non-manifold mesh is refused after
    the sync, and the context then takes a good upload again."""
    m = M.kuhn_cube(72)
    x, t = M.new_points(72)
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, M.velocity)]
    res = []
    for adja in (True, False):
        transfer.upload_background(m, sols, 0, adja=adja)
        transfer.upload_points(x, t)
        transfer.run()
        res.append(transfer.download())
    a, b = res
    assert np.array_equal(a.elem, b.elem) and np.array_equal(a.status, b.status)
    for sa, sb in zip(a.sols, b.sols):
        assert np.array_equal(sa.view(np.int64), sb.view(np.int64))
    bad = M.Mesh(m.xyz, np.concatenate([m.tet, m.tet[1:2]]), None, m.tria, m.adjt, m.hausd)
    with pytest.raises(RuntimeError, match="non-manifold"):
        transfer.upload_background(bad, sols, 0, adja=False)
    with pytest.raises(RuntimeError):
        transfer.run()                                   # no background after a refused upload
    transfer.upload_background(m, sols, 0, adja=False)
    transfer.upload_points(x, t)
    transfer.run()
    c = transfer.download()
    assert np.array_equal(a.elem, c.elem)


def test_non_manifold_reported(transfer):
    m = M.kuhn_cube(3)
    tet = np.concatenate([m.tet, m.tet[1:2]])          # a duplicated tet
    with pytest.raises(RuntimeError, match="non-manifold"):
        transfer.build_adja(tet, m.np)
