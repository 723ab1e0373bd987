"""integration/pmmg_pmx.c -- ParMmg's own seams with their exact reference
signatures (src/parmmg.h:472-473,564-566) over the C ABI -- compiled as C99
against a test-local parmmg.h (tests/c/pmmg_stub/) and driven by
tests/c/adapter_demo.c in the reference's call order of one iteration:
copy (src/libparmmg1.c:792, before any device context exists) -> interp
(:829) -> tetraQual(parmesh, 1) (:845) -> qualhisto OUTQUA (:910) ->
prilen(parmesh, 1, 0) (:964), then the centralized input-side calls
(src/libparmmg.c:175,185); and two iterations with group contexts kept
across them (PMMG_tetraQual on the device-resident new mesh).  Results
against the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

from helpers import bits_equal, compare_volume
from oracle import oracle as O
from parmmg_amd import mesh as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "integration", "pmmg_pmx.c"), os.path.join(ROOT, "tests", "c", "adapter_demo.c")]
BIN = os.path.join(ROOT, "tests", "c", "_build", "adapter_demo")


def build_adapter_demo(extra=()) -> str:
    from parmmg_amd import build
    lib = build.build_transfer()
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    out = BIN + "".join(extra).replace("-", "_").replace("=", "_")
    deps = SRC + [os.path.join(ROOT, "include", "pmx_transfer.h"),
                  os.path.join(ROOT, "tests", "c", "pmmg_stub", "parmmg.h"), lib]
    if not os.path.exists(out) or any(os.path.getmtime(d) > os.path.getmtime(out) for d in deps):
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-O1", *extra,
                        "-I", os.path.join(ROOT, "tests", "c", "pmmg_stub"), "-I", os.path.join(ROOT, "include"),
                        *SRC, "-L", os.path.dirname(lib), "-lpmx_transfer",
                        f"-Wl,-rpath,{os.path.dirname(lib)}", "-o", out], check=True)
    return out


def test_adapter_compiles_as_c():
    """The exact-signature adapter compiles as C99 (-Wall -Wextra -Werror) and
    links against the library (no GPU needed)."""
    assert os.path.exists(build_adapter_demo())


def write_case(d, metric="iso", n=6, n2=7):
    """A background group (Kuhn cube n) and a new mesh (Kuhn cube n2, another
    jitter) in Mmg's layout; a few background vertices MG_REQ (frozen: the new
    mesh keeps them, same index and position) and a few boundary ridge points."""
    old = M.kuhn_cube(n, seed=3)
    new = M.kuhn_cube(n2, seed=4)
    otag = np.zeros(old.np + 1, np.uint16)
    onb = np.any((old.xyz[1:] == 0.0) | (old.xyz[1:] == 1.0), axis=1)
    otag[1:][onb] = M.TAG_BDY
    req = np.arange(1, min(old.np, new.np) + 1, 13)
    otag[req] |= M.TAG_REQ
    ntag = np.zeros(new.np + 1, np.uint16)
    nnb = np.any((new.xyz[1:] == 0.0) | (new.xyz[1:] == 1.0), axis=1)
    ntag[1:][nnb] = M.TAG_BDY
    ntag[1:][nnb & (np.sum((new.xyz[1:] == 0.0) | (new.xyz[1:] == 1.0), axis=1) >= 2)] |= 2   # MG_GEO ridges
    ntag[req] = otag[req]
    nxyz = new.xyz.copy()
    nxyz[req] = old.xyz[req]
    f = M.shock_metric if metric == "ani" else M.iso_metric
    omet = M.on_vertices(old, f)
    ofld = M.on_vertices(old, M.level_set)
    files = dict(old_xyz=old.xyz, old_tet=old.tet, old_tag=otag, old_met=omet, old_fld=ofld,
                 new_xyz=nxyz, new_tet=new.tet, new_tag=ntag)
    for k, a in files.items():
        np.ascontiguousarray(a).tofile(os.path.join(d, k + ".bin"))
    with open(os.path.join(d, "sizes.txt"), "w") as fh:
        fh.write(f"{old.np} {old.ne} {new.np} {new.ne} {omet.shape[1]} {ofld.shape[1]}\n")
    return old, new, otag, ntag, nxyz, omet, ofld, req


def run_demo(d, mode):
    r = subprocess.run([build_adapter_demo(), d, mode], capture_output=True, text=True, timeout=300)
    recs = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    return r, recs


@pytest.mark.gpu
def test_adapter_reference_call_order(tmp_path):
    d = str(tmp_path)
    old, new, otag, ntag, nxyz, omet, ofld, req = write_case(d, "iso")
    r, recs = run_demo(d, "full")
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    assert calls == {"copy": 1, "interp": 1, "tetraqual": 1, "qualhisto_out": 1, "prilen_1_dist": 1,
                     "qualhisto_in": 1, "prilen_0_central": 1}, calls
    met = np.fromfile(os.path.join(d, "out_met.bin")).reshape(new.np + 1, 1)
    fld = np.fromfile(os.path.join(d, "out_fld.bin")).reshape(new.np + 1, 1)
    qual = np.fromfile(os.path.join(d, "out_qual.bin"))
    # frozen points: the old values (the copy), untouched by the interpolation
    assert np.array_equal(met[req], omet[req]) and np.array_equal(fld[req], ofld[req])
    # the interpolation against the oracle: volume points bit-exact or ties
    o = O.Oracle(old)
    x, t = nxyz[1:], ntag[1:]
    outs, elem, st, *_ = o.interp(x, t, [omet, ofld], imet=0)
    from parmmg_amd.transfer import Transfer
    tr = Transfer(0)
    tr.upload_background(old, [omet, ofld], 0)
    tr.upload_points(x, t, tets_mmg=new.tet)
    tr.run()
    g = tr.download()
    tr.close()
    live = (t & M.TAG_REQ) == 0
    assert np.array_equal(g.sols[0][live], met[1:][live]) and np.array_equal(g.sols[1][live], fld[1:][live])
    c = compare_volume(o, x, t, ([met[1:], fld[1:]], g.elem, g.status), (outs, elem, st), [omet, ofld])
    assert c["same"] >= c["nvol"] - 3
    # tetraQual(parmesh, 1) on the new mesh in its interpolated metric:
    # iso, so metRidTyp 1 == 0 (the oracle's MMG3D_tetraQual restatement)
    mesh_new = M.Mesh(nxyz, new.tet, new.adja, new.tria, new.adjt)
    qo = O.tetra_qual(mesh_new, None)
    assert np.array_equal(qual[1:], qo[1:])
    # qualhisto (OUTQUA, nrid from the ridge tags) and prilen vs the oracle
    qh = [c["qualhisto"] for c in recs if "qualhisto" in c]
    pl = [c["prilen"] for c in recs if "prilen" in c]
    assert len(qh) == 2 and len(pl) == 2
    ref_out = O.qualhisto(mesh_new, qo, tags=ntag)
    ref_in = O.qualhisto(mesh_new, qo)
    for got, ref in ((qh[0], ref_out), (qh[1], ref_in)):
        for k in ("ne", "good", "med", "his", "nrid"):
            assert got[k] == (list(ref[k]) if k == "his" else ref[k]), (k, got[k], ref[k])
        assert got["min"] == ref["min"] and got["max"] == ref["max"]
        assert abs(got["avg"] - ref["avg"]) <= 1e-12 * abs(ref["avg"])
    lo = O.prilen(mesh_new, met, tags=ntag)
    for p in pl:
        assert p["ned"] == lo["ned"] and p["nullEdge"] == lo["nullEdge"]
        assert p["hl"] == lo["hl"]                      # glibc's log1p restated on the device (r06)
        assert p["lmin"] == pytest.approx(lo["lmin"], rel=1e-15) and p["lmax"] == pytest.approx(lo["lmax"], rel=1e-15)


@pytest.mark.gpu
def test_adapter_ani_ridge_metric(tmp_path):
    """metRidTyp = 1 with an anisotropic metric (Mmg's ridge metric storage):
    PMMG_tetraQual(parmesh,1) (src/libparmmg1.c:845) runs on the device-resident
    new mesh and equals the oracle's MMG5_caltet_ani restatement (the mean
    metric without the non-singular ridge points, from the new points' tags)
    bit for bit; metRidTyp = 0 equals MMG5_caltet33_ani.  PMMG_prilen(parmesh,1,0)
    (:964) -- ParMmg's output call -- measures the new mesh's edges in its
    interpolated tensor metric along the curved surface (the mesh's xTetra
    edge tags and point / xPoint normals, read in place by the binding,
    MMG5_lenedg_ani) and PMMG_prilen(parmesh,0,1) (src/libparmmg.c:185) in
    classic storage (MMG5_lenedg33_ani): both equal the oracle's restatement
    bit for bit."""
    from helpers import cube_surface
    d = str(tmp_path)
    old, new, otag, ntag, nxyz, omet, ofld, req = write_case(d, "ani")
    stag, surf, _ = cube_surface(new, noise=0.08)
    for k, a in dict(new_xt=surf["xt"].astype(np.int32), new_xtag=surf["xtag"].astype(np.uint16),
                     new_pn=surf["n"], new_xp=surf["xp"].astype(np.int32), new_n1=surf["n1"],
                     new_n2=surf["n2"]).items():
        np.ascontiguousarray(a).tofile(os.path.join(d, k + ".bin"))
    with open(os.path.join(d, "surf_sizes.txt"), "w") as fh:
        fh.write(f"{surf['xtag'].shape[0] - 1} {surf['n1'].shape[0] - 1}\n")
    r, recs = run_demo(d, "ani")
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    assert calls["tetraqual_ani_1"] == 1 and calls["tetraqual_ani_0"] == 1, calls
    assert calls["prilen_ani_1"] == 1 and calls["prilen_ani_0_central"] == 1, (calls, r.stderr)
    met = np.fromfile(os.path.join(d, "out_met.bin")).reshape(new.np + 1, 6)
    mesh_new = M.Mesh(nxyz, new.tet, new.adja, new.tria, new.adjt)
    pl = [c["prilen"] for c in recs if "prilen" in c]
    assert len(pl) == 2
    for got, mrt in zip(pl, (1, 0)):
        ref = O.prilen(mesh_new, met, tags=ntag, met_rid_typ=mrt, surface=surf)
        for k in ("ned", "nullEdge", "amin", "bmin", "amax", "bmax", "hl", "lmin", "lmax"):
            assert got[k] == ref[k], (mrt, k, got[k], ref[k])
    q1 = np.fromfile(os.path.join(d, "out_qual_ani1.bin"))
    q0 = np.fromfile(os.path.join(d, "out_qual_ani0.bin"))
    o1 = O.tetra_qual(mesh_new, met, tags=ntag, met_rid_typ=1)
    o0 = O.tetra_qual(mesh_new, met)
    assert np.array_equal(q1[1:], o1[1:]) and np.array_equal(q0[1:], o0[1:])
    assert np.count_nonzero(q1[1:] != q0[1:]) > 0       # the ridge points change the mean


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["nolocate", "hsiz_nofield"])
def test_adapter_quality_when_nothing_located(tmp_path, mode):
    """A group whose interpolation locates nothing (src/interpmesh_pmmg.c:
    497-512: no input metric and no field, or -hsiz and no field) keeps no
    step on its context: PMMG_tetraQual (src/libparmmg1.c:845) must then take
    the upload path and still set every valid tet's quality (the r04 advisor's
    finding: the binding had marked every group resident)."""
    d = str(tmp_path)
    old, new, otag, ntag, nxyz, omet, ofld, req = write_case(d, "iso")
    r, recs = run_demo(d, mode)
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    assert calls == {"interp": 1, "tetraqual": 1}, (calls, r.stderr)
    qual = np.fromfile(os.path.join(d, "out_qual.bin"))
    mesh_new = M.Mesh(nxyz, new.tet, new.adja, new.tria, new.adjt)
    assert np.array_equal(qual[1:], O.tetra_qual(mesh_new, None)[1:])
    met = np.fromfile(os.path.join(d, "out_met.bin"))
    assert np.all(met[1:] == 0.05)                 # Mmg's metric, or the constant size


@pytest.mark.gpu
def test_adapter_refuses_optimles(tmp_path):
    """mesh->info.optimLES (a run-time flag, src/quality_pmmg.c:221-224):
    MMG3D_computeLESqua is not restated, PMMG_qualhisto fails loudly."""
    d = str(tmp_path)
    write_case(d, "iso")
    r, recs = run_demo(d, "refuse_les")
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    assert calls["qualhisto_les"] == 0
    assert "optimLES" in r.stderr


@pytest.mark.gpu
def test_adapter_two_iterations_resident_quality(tmp_path):
    """Two ParMmg iterations through the adapter (src/libparmmg1.c:653-845):
    iteration 2 has two groups, each on the group context kept from iteration
    1.  PMMG_tetraQual right after the interpolation runs on the device-resident
    new mesh (only the metric rows the step did not write cross PCIe); it must
    equal the re-upload path bit for bit, and the oracle's MMG3D_tetraQual.
    Group 0's background is iteration 1's result (PMMG_update_oldGrps); its
    interpolation must equal a direct step on that background; group 1 repeats
    iteration 1's inputs and must reproduce its results bit for bit."""
    d = str(tmp_path)
    # new meshes on the background's lattice: a frozen point keeps its index
    # and moves by less than the jitter, so iteration 1's new mesh -- the
    # background of iteration 2 -- stays untangled (in a tangled background a
    # point can lie in several overlapping tets and the answer depends on the
    # walk)
    old, new, otag, ntag, nxyz, omet, ofld, req = write_case(d, "iso", n=6, n2=6)
    # iteration 2's new mesh keeps the frozen points of its background
    # (iteration 1's new mesh): same index, same position, MG_REQ
    new2 = M.kuhn_cube(6, seed=9)
    ntag2 = np.zeros(new2.np + 1, np.uint16)
    nb2 = np.any((new2.xyz[1:] == 0.0) | (new2.xyz[1:] == 1.0), axis=1)
    ntag2[1:][nb2] = M.TAG_BDY
    ntag2[req] = ntag[req]
    xyz2 = new2.xyz.copy()
    xyz2[req] = nxyz[req]
    for k, a in dict(new2_xyz=xyz2, new2_tet=new2.tet, new2_tag=ntag2).items():
        np.ascontiguousarray(a).tofile(os.path.join(d, k + ".bin"))
    with open(os.path.join(d, "sizes2.txt"), "w") as fh:
        fh.write(f"{new2.np} {new2.ne}\n")
    r, recs = run_demo(d, "iterate")
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    assert calls == {"copy": 1, "interp": 1, "tetraqual_1_res": 1, "tetraqual_1_upl": 1, "interp2": 1,
                     "tetraqual_2_res": 1, "tetraqual_2_upl": 1, "prilen_2grp": 0}, calls

    def rd(name, shape=None):
        a = np.fromfile(os.path.join(d, name))
        return a if shape is None else a.reshape(shape)
    # resident quality == re-upload quality, every group of both iterations
    for tag in ("1_", "2a", "2b"):
        qr, qu = rd(f"out_q{tag}_res.bin"), rd(f"out_q{tag}_upl.bin")
        assert qr.view(np.int64)[1:].tolist() == qu.view(np.int64)[1:].tolist(), tag
    mesh1 = M.Mesh(nxyz, new.tet, new.adja, new.tria, new.adjt)
    qo = O.tetra_qual(mesh1, None)
    assert np.array_equal(rd("out_q1__res.bin")[1:], qo[1:])
    assert np.array_equal(rd("out_q2b_res.bin")[1:], qo[1:])
    mesh2 = M.Mesh(xyz2, new2.tet, new2.adja, new2.tria, new2.adjt)
    assert np.array_equal(rd("out_q2a_res.bin")[1:], O.tetra_qual(mesh2, None)[1:])
    # group 1 of iteration 2 = iteration 1 (same inputs, its own context)
    assert np.array_equal(rd("out2b_met.bin"), rd("out_met.bin"))
    assert np.array_equal(rd("out2b_fld.bin"), rd("out_fld.bin"))
    # group 0: a direct step on iteration 1's result as background
    bgm, bgf = rd("bg2_met.bin", (new.np + 1, 1)), rd("bg2_fld.bin", (new.np + 1, 1))
    from parmmg_amd.transfer import Transfer
    tr = Transfer(0)
    # the background's boundary trias numbered as the driver's snapshot builds
    # them (pmx_build_adja / pmx_build_bdry; the surface walk depends on it)
    adja1 = tr.build_adja(new.tet, new.np)
    tria1, adjt1 = tr.build_bdry(new.tet, new.np, adja1)
    tr.upload_background(M.Mesh(nxyz, new.tet, adja1, tria1, adjt1), [bgm, bgf], 0)
    tr.upload_points(xyz2[1:], ntag2[1:], tets_mmg=new2.tet)
    tr.run()
    g = tr.download()
    tr.close()
    m2, f2 = rd("out2_met.bin", (new2.np + 1, 1)), rd("out2_fld.bin", (new2.np + 1, 1))
    live = (ntag2[1:] & M.TAG_REQ) == 0
    for a, b in ((g.sols[0], m2[1:]), (g.sols[1], f2[1:])):
        bad = np.nonzero(live & ~bits_equal(a, b))[0]
        assert len(bad) == 0, (bad[:10], a[bad[:10], 0], b[bad[:10], 0], ntag2[1:][bad[:10]], g.elem[bad[:10]])
    # its frozen points: the background's values (PMMG_copyMetricsAndFields_point)
    assert np.array_equal(m2[req], bgm[req]) and np.array_equal(f2[req], bgf[req])


def _twoproc(d, which):
    r, recs = run_demo(d, "twoproc_" + which)
    assert r.returncode == 0, r.stdout + r.stderr
    calls = {c["call"]: c["ret"] for c in recs if "call" in c}
    mpi = [c for c in recs if "mpi" in c]
    return calls, mpi, r


@pytest.mark.parametrize("which", ["prilen", "qualhisto"])
def test_adapter_two_ranks_agree_on_failure_cpu(tmp_path, which):
    """Two ranks (forked processes, a socketpair MPI shim) through the
    statistics seams; without a device both fail locally: each reaches the
    agreement (one MPI_Allreduce MIN) and returns 0 -- neither waits in a
    collective the other skipped (the r03 advisor's finding)."""
    d = str(tmp_path)
    write_case(d, "iso")
    calls, mpi, r = _twoproc(d, which)
    assert calls == {f"{which}_rank0": 0, f"{which}_rank1": 0}
    assert sorted((m["mpi"], m["rank"]) for m in mpi) == [("allreduce", 0), ("allreduce", 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["prilen", "qualhisto"])
def test_adapter_two_ranks_agree_on_failure(tmp_path, which):
    """The same on the GPU, where rank 0 succeeds locally and rank 1 fails
    (prilen: two groups, the reference's refusal at src/quality_pmmg.c:623-627;
    qualhisto: an upload it must refuse): both return 0 after the agreement,
    and no rank enters the RCCL set-up (no MPI_Bcast of its id)."""
    d = str(tmp_path)
    write_case(d, "iso")
    calls, mpi, r = _twoproc(d, which)
    assert calls == {f"{which}_rank0": 0, f"{which}_rank1": 0}
    assert sorted((m["mpi"], m["rank"], m.get("value")) for m in mpi) == [("allreduce", 0, 0), ("allreduce", 1, 0)]
