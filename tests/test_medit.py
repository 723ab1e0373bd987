"""Medit I/O of the C library (pmx_medit_*; CPU only, no GPU call).

ParMmg reads and writes its meshes and solutions through Mmg (reference
src/inout_pmmg.c:440-991).  The ASCII reader is checked against the
reference's own libexamples fixtures (tests/golden/ref_inputs, copied data
files) and the Python reader; ASCII and binary writers round-trip bit for bit.
Binary files: the format is restated from the public libMeshb description
(no binary file in the reference: parity unpinned); hand-assembled files of
versions 1-4 check the reader's widths and block positions.
"""
import os
import struct

import numpy as np
import pytest

from conftest import REF_INPUTS
from parmmg_amd import medit as MD
from parmmg_amd import mesh as M


def _tokens(path):
    with open(path) as f:
        return f.read().split()


@pytest.mark.parametrize("name", ["cube.mesh", "wave.0.mesh"])
def test_reference_meshes_read(name):
    path = os.path.join(REF_INPUTS, name)
    m = MD.read_mesh(path)
    ref = M.read_medit(path)
    assert np.array_equal(m.xyz, ref.xyz) and np.array_equal(m.tet, ref.tet)
    tok = _tokens(path)
    if "Triangles" in tok:
        i = tok.index("Triangles")
        n = int(tok[i + 1])
        a = np.array(tok[i + 2: i + 2 + 4 * n], np.int64).reshape(n, 4)
        assert np.array_equal(m.tria[1:], a[:, :3]) and np.array_equal(m.triaref[1:], a[:, 3])
    i = tok.index("Vertices")
    n = int(tok[i + 1])
    refs = np.array(tok[i + 2: i + 2 + 4 * n], np.float64).reshape(n, 4)[:, 3]
    assert np.array_equal(m.vref[1:], refs.astype(np.int32))
    assert np.array_equal(m.required, M.read_medit_required(path).astype(np.int32))


@pytest.mark.parametrize("name", ["cube-met.sol", "cube-solphys.sol"])
def test_reference_solutions_read(name):
    path = os.path.join(REF_INPUTS, name)
    got = MD.read_sol(path)
    ref = M.read_medit_sol(path)
    assert len(got) == len(ref)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


def _case():
    m = M.kuhn_cube(4, seed=3)
    rng = np.random.default_rng(0)
    vref = rng.integers(0, 5, m.np + 1).astype(np.int32)
    tetref = rng.integers(0, 3, m.ne + 1).astype(np.int32)
    triaref = rng.integers(1, 7, m.nt + 1).astype(np.int32)
    vref[0] = tetref[0] = triaref[0] = 0
    req = np.array([1, 5, 17, m.np], np.int32)
    sols = [M.on_vertices(m, M.iso_metric), M.on_vertices(m, M.velocity), M.on_vertices(m, M.shock_metric)]
    return m, vref, tetref, triaref, req, sols


@pytest.mark.parametrize("ext", ["mesh", "meshb"])
def test_mesh_round_trip(tmp_path, ext):
    m, vref, tetref, triaref, req, _ = _case()
    p = str(tmp_path / f"a.{ext}")
    MD.write_mesh(p, m.xyz, m.tet, m.tria, req, vref, tetref, triaref)
    r = MD.read_mesh(p)
    assert np.array_equal(r.xyz.view(np.int64)[1:], m.xyz.view(np.int64)[1:])   # bitwise
    assert np.array_equal(r.tet[1:], m.tet[1:]) and np.array_equal(r.tria[1:], m.tria[1:])
    assert np.array_equal(r.vref, vref) and np.array_equal(r.tetref, tetref)
    assert np.array_equal(r.triaref, triaref) and np.array_equal(r.required, req)
    # the Python ASCII reader agrees on the C writer's file
    if ext == "mesh":
        assert np.array_equal(M.read_medit(p).tet, m.tet)


@pytest.mark.parametrize("ext", ["sol", "solb"])
def test_sol_round_trip(tmp_path, ext):
    m, *_, sols = _case()
    p = str(tmp_path / f"a.{ext}")
    MD.write_sol(p, sols)
    got = MD.read_sol(p)
    for a, b in zip(got, sols):
        assert np.array_equal(a[1:].view(np.int64), b[1:].view(np.int64))
    if ext == "sol":                       # tensor order: the Python reader/writer agree
        for a, b in zip(M.read_medit_sol(p), sols):
            assert np.array_equal(a[1:], b[1:])
        q = str(tmp_path / "py.sol")
        M.write_medit_sol(q, sols)
        for a, b in zip(MD.read_sol(q), sols):
            assert np.array_equal(a[1:], b[1:])


def _meshb(ver, xyz, tets, extra_block=True):
    """Hand-assembled .meshb of a given version (positions patched)."""
    ip = "<q" if ver >= 3 else "<i"          # next-block positions
    cnt = "<q" if ver == 4 else "<i"         # counts
    it = "q" if ver == 4 else "i"
    rl = "f" if ver == 1 else "d"
    out = bytearray(struct.pack("<ii", 1, ver))

    def block(kw, body, count=None):
        out.extend(struct.pack("<i", kw))
        at = len(out)
        out.extend(struct.pack(ip, 0))
        if count is not None:
            out.extend(struct.pack(cnt, count))
        out.extend(body)
        struct.pack_into(ip, out, at, len(out))

    block(3, struct.pack("<i", 3))
    if extra_block:                          # an unknown keyword (Corners) is skipped
        block(13, struct.pack("<" + it * 2, 1, 2), 2)
    block(4, b"".join(struct.pack("<" + rl * 3 + it, *p, 7) for p in xyz), len(xyz))
    block(8, b"".join(struct.pack("<" + it * 5, *t, 2) for t in tets), len(tets))
    out.extend(struct.pack("<i", 54))
    out.extend(struct.pack(ip, 0))
    return bytes(out)


@pytest.mark.parametrize("ver", [1, 2, 3, 4])
def test_meshb_versions(tmp_path, ver):
    xyz = [(0.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0), (0.1, 0.2, 0.3)]
    tets = [(1, 2, 3, 4), (2, 3, 4, 5)]
    p = tmp_path / "v.meshb"
    p.write_bytes(_meshb(ver, xyz, tets))
    r = MD.read_mesh(str(p))
    want = np.array(xyz, np.float32 if ver == 1 else np.float64).astype(np.float64)
    assert r.version == ver
    assert np.array_equal(r.xyz[1:], want) and np.all(r.vref[1:] == 7)
    assert np.array_equal(r.tet[1:], np.array(tets)) and np.all(r.tetref[1:] == 2)


def test_errors_are_reported(tmp_path):
    with pytest.raises(RuntimeError, match="cannot open"):
        MD.read_mesh(str(tmp_path / "missing.mesh"))
    p = tmp_path / "bad.meshb"
    p.write_bytes(struct.pack("<ii", 0x01000000, 2))
    with pytest.raises(RuntimeError, match="native-endian"):
        MD.read_mesh(str(p))
    q = tmp_path / "t.mesh"
    q.write_text("MeshVersionFormatted 2\nDimension 3\nVertices\n3\n0 0 0 0\n1 1\n")
    with pytest.raises(RuntimeError, match="truncated"):
        MD.read_mesh(str(q))
