"""Host-side mirror of ParMmg's transfer interface, over the C ABI.

Names and argument meaning follow the reference:

* :meth:`Transfer.interp_metrics_and_fields` -- ``PMMG_interpMetricsAndFields``
  (reference src/interpmesh_pmmg.c:663-741), one call per remesh iteration,
  groups are independent.
* :meth:`Transfer.copy_metrics_and_fields_point` --
  ``PMMG_copyMetricsAndFields_point`` (src/interpmesh_pmmg.c:432-446).
* :meth:`Transfer.tetra_qual`, :meth:`Transfer.qualhisto`,
  :meth:`Transfer.prilen` -- ``PMMG_tetraQual`` / ``PMMG_qualhisto`` /
  ``PMMG_prilen`` (src/quality_pmmg.c).

Errors follow the reference's 1/0 convention at the C ABI and surface here as
``RuntimeError`` with ``pmx_last_error``.  Everything runs on the GPU; there is
no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from . import _native as N
from .mesh import Mesh


def _dp(a):
    return a.ctypes.data_as(N.dptr) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(N.iptr) if a is not None else None


def _shift(a, rec: int, ctype):
    """Pointer to record -1 of a 0-based array: a 1-based view (the library
    only dereferences records first..last >= 1)."""
    return C.cast(C.c_void_p(a.ctypes.data - rec), C.POINTER(ctype))


def _tets_1based(tets) -> np.ndarray:
    """0-based new tets (v[0] < 0: deleted) -> Mmg's 1-based records (v[0] = 0)."""
    tv = np.ascontiguousarray(tets, np.int32) + 1
    tv[tv[:, 0] < 0, 0] = 0
    tv[0] = 0
    return tv


def mesh_view(m: Mesh) -> N.MeshView:
    v = N.MeshView()
    v.np, v.ne, v.nt = m.np, m.ne, m.nt
    v.point_c = _dp(m.xyz)
    v.point_stride = 3 * 8
    v.tetra_v = _ip(m.tet)
    v.tetra_stride = 4 * 4
    v.adja = _ip(m.adja)
    v.tria_v = _ip(m.tria) if m.nt > 0 else None
    v.tria_stride = 3 * 4
    v.adjt = _ip(m.adjt) if m.nt > 0 else None
    v.hausd = m.hausd
    return v


@dataclasses.dataclass
class Result:
    sols: list            # per solution: (npts, size) arrays
    elem: np.ndarray      # located tet (volume) / tria (surface), 1-based
    status: np.ndarray    # 1 found, -1 found by exhaustive search, 0 closest
    steps: np.ndarray


class Transfer:
    """One device context (one GPU).  ``device`` = rank % ndev in ParMmg terms."""

    def __init__(self, device: int = 0):
        self.lib = N.load()
        self.ctx = self.lib.pmx_create(device)
        if not self.ctx:
            raise RuntimeError("pmx_create failed (no HIP device visible)")
        self._keep = []
        self.sizes: list[int] = []
        self.npts = 0
        self.n_new_tets = 0

    def close(self):
        if self.ctx:
            self.lib.pmx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, r: int, what: str):
        if not r:
            raise RuntimeError(f"{what}: {self.lib.pmx_last_error(self.ctx).decode()}")

    def device_info(self) -> str:
        buf = C.create_string_buffer(256)
        self._chk(self.lib.pmx_device_info(self.ctx, buf, 256), "pmx_device_info")
        return buf.value.decode()

    def set_stream(self, stream_ptr: int | None):
        self._chk(self.lib.pmx_set_stream(self.ctx, C.c_void_p(stream_ptr or 0)), "pmx_set_stream")

    def synchronize(self):
        self._chk(self.lib.pmx_synchronize(self.ctx), "pmx_synchronize")

    # ---- device-resident interface ------------------------------------------
    def upload_background(self, m: Mesh, sols: list[np.ndarray], imet: int = 0, adja: bool = True):
        """sols: (np+1, size) arrays in Mmg layout; imet: index of the metric or -1.
        adja=False: Mmg's adjacency is not sent; the device rebuilds it from the
        connectivity (16 B/tet less over PCIe, face matching overlapped with
        the rest of the upload)."""
        arr = [np.ascontiguousarray(s, np.float64) for s in sols]
        views = (N.SolView * max(len(arr), 1))()
        for i, a in enumerate(arr):
            views[i].size = a.shape[1] if a.ndim == 2 else 1
            views[i].m = _dp(a)
        mv = mesh_view(m)
        if not adja:
            mv.adja = None
        self._chk(self.lib.pmx_upload_background(self.ctx, C.byref(mv), len(arr), views,
                                                 imet if arr else -1), "pmx_upload_background")
        self.sizes = [v.size for v in views[: len(arr)]]

    def copy_required(self, perm: np.ndarray | None = None, copy_metric: bool = True):
        """pmx_copy_required: frozen (MG_REQ) background points' values into the
        unwritten rows of the last step's results; perm: (np+1,) permNodGlob
        (1-based new point of background vertex ip)."""
        pp = None if perm is None else np.ascontiguousarray(perm, np.int32)
        self._chk(self.lib.pmx_copy_required(self.ctx, _ip(pp), int(copy_metric)), "pmx_copy_required")

    def set_residency(self, on: bool = True):
        self._chk(self.lib.pmx_set_residency(self.ctx, int(on)), "pmx_set_residency")

    def upload_points(self, xyz: np.ndarray, tags: np.ndarray | None = None,
                      tets: np.ndarray | None = None, tets_mmg: np.ndarray | None = None):
        """xyz: (n, 3) new points (0-based list); tags: MMG5_Point.tag values;
        tets: optional (ne+1, 4) new tets with 0-based point indices in rows
        1..ne -- only points of valid tets (v[0] >= 0 here) are located.
        The C view is Mmg's 1-based one (points 1..n, a tet valid when
        v[0] > 0), so the pointers are shifted by one record.  tets_mmg: the
        same tets already in that layout (1-based, v[0] = 0 deleted; passed
        as is, as a C caller would)."""
        xyz = np.ascontiguousarray(xyz, np.float64)
        pv = N.PointsView()
        pv.first, pv.last = 1, xyz.shape[0]
        pv.c, pv.stride = _shift(xyz, 24, C.c_double), 24
        self._keep = []
        if tags is not None:
            t = np.ascontiguousarray(tags, np.uint16)
            self._keep.append(t)
            pv.tag, pv.tag_stride = _shift(t, 2, C.c_uint16), 2
        if tets is not None or tets_mmg is not None:
            tv = _tets_1based(tets) if tets_mmg is None else np.ascontiguousarray(tets_mmg, np.int32)
            self._keep.append(tv)
            pv.tetra_v, pv.tetra_stride, pv.ne = _ip(tv), 16, tv.shape[0] - 1
        self._chk(self.lib.pmx_upload_points(self.ctx, C.byref(pv)), "pmx_upload_points")
        self.npts = xyz.shape[0]
        # the view's tets are the device's new tets (read by the first run):
        # new_mesh_qual(None) sizes its output by them
        self.n_new_tets = int(pv.ne) if pv.tetra_v else 0

    def run(self, hsiz: float = 0.0, timing: bool = False, max_walk: int = 0, hint_stride: int = 0,
            flags: int = 0, record_starts: bool = False):
        """One step (asynchronous; device-side failures surface in
        synchronize()/download()).  flags: ``_native.RUN_*``.  record_starts:
        keep every volume point's walk start tet for starts() (diagnostics;
        the production step does not write it)."""
        if record_starts:
            flags |= N.RUN_RECORD_STARTS
        o = N.RunOpts()
        o.hsiz, o.timing, o.max_walk, o.hint_stride, o.flags = hsiz, int(timing), max_walk, hint_stride, flags
        self._chk(self.lib.pmx_run(self.ctx, C.byref(o)), "pmx_run")

    def download(self, init: list[np.ndarray] | None = None, into: Result | None = None,
                 sols_only: bool = False) -> Result:
        """Results into new arrays (``init`` = values kept where a field is not
        written), or in place into the arrays of ``into`` -- ParMmg's case, whose
        ``met->m`` / ``field->m`` already exist (no allocation per step).
        sols_only: the fields only (what PMMG_interpMetricsAndFields returns;
        elem/status/steps are not copied)."""
        n = self.npts
        if into is not None:
            outs, elem, status, steps = into.sols, into.elem, into.status, into.steps
            if (len(outs) != len(self.sizes) or any(
                    a.dtype != np.float64 or not a.flags.c_contiguous or a.shape != (n, sz)
                    for a, sz in zip(outs, self.sizes)) or any(
                    a.dtype != np.int32 or not a.flags.c_contiguous or a.shape != (n,)
                    for a in (elem, status, steps))):
                raise ValueError("download(into=...): arrays do not match the uploaded step")
        else:
            outs = []
            for i, sz in enumerate(self.sizes):
                outs.append(np.array(init[i], np.float64, copy=True).reshape(n, sz) if init is not None
                            else np.full((n, sz), np.nan))
            elem = np.zeros(n, np.int32)
            status = np.zeros(n, np.int32)
            steps = np.zeros(n, np.int32)
        views = (N.SolView * max(len(self.sizes), 1))()
        for i, (a, sz) in enumerate(zip(outs, self.sizes)):
            views[i].size, views[i].m = sz, _dp(a)
        if sols_only:
            self._chk(self.lib.pmx_download(self.ctx, views, n, None, None, None), "pmx_download")
        else:
            self._chk(self.lib.pmx_download(self.ctx, views, n, _ip(elem), _ip(status), _ip(steps)),
                      "pmx_download")
        return Result(outs, elem, status, steps)

    def starts(self) -> np.ndarray:
        s = np.zeros(self.npts, np.int32)
        self._chk(self.lib.pmx_download_starts(self.ctx, _ip(s), len(s)), "pmx_download_starts")
        return s

    def border(self) -> tuple[np.ndarray, np.ndarray]:
        e = np.zeros(self.npts, np.int32)
        v = np.zeros(self.npts, np.int32)
        self._chk(self.lib.pmx_download_border(self.ctx, _ip(e), _ip(v), len(e)), "pmx_download_border")
        return e, v

    def locate_stats(self) -> dict:
        st = N.LocateStats()
        self._chk(self.lib.pmx_locate_stats_get(self.ctx, C.byref(st)), "pmx_locate_stats_get")
        return {f: getattr(st, f) for f, _ in N.LocateStats._fields_}

    def seq_surface_stats(self) -> dict:
        """After a RUN_SEQUENTIAL_SURFACE step: the surface sequence length and
        the queries replayed one by one on the reference's state."""
        a, b = C.c_int64(), C.c_int64()
        self._chk(self.lib.pmx_seq_surface_stats(self.ctx, C.byref(a), C.byref(b)), "pmx_seq_surface_stats")
        return {"nseq": a.value, "nreplay": b.value}

    def seq_volume_stats(self) -> dict:
        """After a RUN_SEQUENTIAL_VOLUME step: the volume sequence length and
        the walks replayed one by one on the reference's tet flags."""
        a, b = C.c_int64(), C.c_int64()
        self._chk(self.lib.pmx_seq_volume_stats(self.ctx, C.byref(a), C.byref(b)), "pmx_seq_volume_stats")
        return {"nseq": a.value, "nreplay": b.value}

    def wave_stats(self, path: int = 0) -> dict:
        """Lane utilisation of the last step's walks (path 0 volume, 1 surface):
        step_sum / lane_steps, lane_steps = sum over waves of 64 x the wave's
        longest walk; wave_max_hist = waves by their longest walk."""
        st = N.WaveStats()
        self._chk(self.lib.pmx_locate_wave_stats(self.ctx, path, C.byref(st)), "pmx_locate_wave_stats")
        d = {f: getattr(st, f) for f, _ in N.WaveStats._fields_}
        d["wave_max_hist"] = list(st.wave_max_hist)
        d["lane_utilization"] = st.step_sum / st.lane_steps if st.lane_steps else None
        d["mean_wave_max"] = st.lane_steps / 64 / st.waves if st.waves else None
        return d

    def kernel_ms(self, which: int) -> float:
        return self.lib.pmx_kernel_ms(self.ctx, which)

    def timing_reset(self):
        self.lib.pmx_timing_reset(self.ctx)

    def device_buffer(self, which: int) -> int:
        return self.lib.pmx_device_buffer(self.ctx, which) or 0

    # ---- background topology (MMG3D_hashTetra, MMG5_chkBdryTria + hashTria) --
    def build_adja(self, tet: np.ndarray, np_: int) -> np.ndarray:
        """Tet face adjacency on the device, Mmg layout (4*ne+5 ints)."""
        t = np.ascontiguousarray(tet, np.int32)
        ne = t.shape[0] - 1
        adja = np.zeros(4 * ne + 5, np.int32)
        self._chk(self.lib.pmx_build_adja(self.ctx, ne, np_, t.ctypes.data, 16, adja.ctypes.data),
                  "pmx_build_adja")
        return adja

    def build_bdry(self, tet: np.ndarray, np_: int, adja: np.ndarray):
        """Boundary trias ((nt+1, 3), row 0 unused) and their adjacency."""
        t = np.ascontiguousarray(tet, np.int32)
        a = np.ascontiguousarray(adja, np.int32)
        ne = t.shape[0] - 1
        maxnt = 4 * ne
        tria = np.zeros((maxnt + 1, 3), np.int32)
        adjt = np.zeros(3 * maxnt + 4, np.int32)
        nt = self.lib.pmx_build_bdry(self.ctx, ne, np_, t.ctypes.data, 16, a.ctypes.data,
                                     tria.ctypes.data, maxnt, adjt.ctypes.data)
        if nt < 0:
            raise RuntimeError(f"pmx_build_bdry: {self.lib.pmx_last_error(self.ctx).decode()}")
        return np.ascontiguousarray(tria[: nt + 1]), np.ascontiguousarray(adjt[: 3 * nt + 4])

    def topo_ms(self) -> float:
        return self.lib.pmx_topo_ms(self.ctx)

    # ---- reference-shaped entry points --------------------------------------
    def interp_metrics_and_fields(self, groups: list[dict], input_met: int = 1,
                                  perm_nod_glob: np.ndarray | None = None) -> int:
        """PMMG_interpMetricsAndFields over ``groups``; each group is a dict with
        keys ``old_mesh`` (Mesh), ``old_met`` ((np+1,size) or None),
        ``old_fields`` (list), ``xyz`` (new points, (np+1,3) Mmg layout),
        ``tags`` (uint16, np+1), ``met`` / ``fields`` (output arrays in Mmg
        layout, written in place), ``hsiz``, optionally ``tets`` (the new
        tets, (ne+1, 4) in Mmg's 1-based layout: the orphan rule and, with
        PMX_SEQUENTIAL set, the reference's visit order)."""
        keep = []
        G = (N.Group * len(groups))()
        for g, d in zip(G, groups):
            xyz = np.ascontiguousarray(d["xyz"], np.float64)
            tags = np.ascontiguousarray(d["tags"], np.uint16)
            keep += [xyz, tags]
            g.points.first, g.points.last = 1, xyz.shape[0] - 1
            g.points.c, g.points.stride = _dp(xyz), 24
            g.points.tag, g.points.tag_stride = tags.ctypes.data_as(N.u16ptr), 2
            if d.get("tets") is not None:             # Mmg layout: (ne+1, 4), 1-based, v[0] = 0 deleted
                tv = np.ascontiguousarray(d["tets"], np.int32)
                keep.append(tv)
                g.points.tetra_v, g.points.tetra_stride, g.points.ne = _ip(tv), 16, tv.shape[0] - 1
            g.hsiz = d.get("hsiz", 0.0)
            om = mesh_view(d["old_mesh"])
            keep.append(om)
            g.old_mesh = om

            def sv(a):
                v = N.SolView()
                v.size, v.m = a.shape[1], _dp(a)
                return v
            if d.get("met") is not None and d.get("old_met") is not None:
                g.met = C.pointer(sv(d["met"]))
                g.old_met = C.pointer(sv(d["old_met"]))
                keep += [g.met, g.old_met]
            fl = d.get("fields") or []
            ofl = d.get("old_fields") or []
            g.nsols = len(fl)
            if fl:
                fa = (N.SolView * len(fl))(*[sv(a) for a in fl])
                ofa = (N.SolView * len(ofl))(*[sv(a) for a in ofl])
                keep += [fa, ofa]
                g.fields = C.cast(fa, C.POINTER(N.SolView))
                g.old_fields = C.cast(ofa, C.POINTER(N.SolView))
        perm = None
        if perm_nod_glob is not None:
            perm = np.ascontiguousarray(perm_nod_glob, np.int32)
        return self.lib.PMX_interpMetricsAndFields(self.ctx, len(groups), G, _ip(perm), input_met)

    # ---- statistics -----------------------------------------------------------
    def upload_point_tags(self, tags: np.ndarray | None):
        """MMG5_Point.tag of the uploaded background, (np+1,) (ridge points for
        the length filter and OUTQUA's nrid)."""
        t = None if tags is None else np.ascontiguousarray(tags, np.uint16)
        self._keep_tags = t
        self._chk(self.lib.pmx_upload_point_tags(self.ctx, t.ctypes.data_as(N.u16ptr) if t is not None
                                                 else None, 2), "pmx_upload_point_tags")

    def tetra_qual(self, ne: int, met_rid_typ: int = 0) -> np.ndarray:
        """MMG3D_tetraQual(mesh, met, metRidTyp) of the uploaded group."""
        q = np.zeros(ne + 1)
        self._chk(self.lib.pmx_tetra_qual(self.ctx, met_rid_typ, _dp(q), len(q)), "pmx_tetra_qual")
        return q

    def count_nodes(self, idx_ip=None, idx_comm=None, intvalues=None, base: int = 1) -> int:
        """PMMG_count_nodes_par on the uploaded group; intvalues is updated in place."""
        n_grp = 0 if idx_ip is None else len(idx_ip)
        ip = np.ascontiguousarray(idx_ip if idx_ip is not None else [], np.int32)
        ic = np.ascontiguousarray(idx_comm if idx_comm is not None else [], np.int32)
        iv = intvalues if intvalues is not None else np.zeros(0, np.int32)
        assert iv.dtype == np.int32 and iv.flags.c_contiguous
        out = C.c_int64()
        self._chk(self.lib.pmx_count_nodes(self.ctx, _ip(ip), _ip(ic), n_grp, _ip(iv), len(iv), base,
                                           C.byref(out)), "pmx_count_nodes")
        return out.value

    @staticmethod
    def _qdict(st) -> dict:
        d = {f: getattr(st, f) for f, _ in N.QualStats._fields_}
        d["his"] = list(st.his)
        return d

    @staticmethod
    def _ldict(st) -> dict:
        d = {f: getattr(st, f) for f, _ in N.LenStats._fields_}
        d["hl"] = list(st.hl)
        return d

    def qualhisto(self, opt: int = N.INQUA) -> dict:
        st = N.QualStats()
        self._chk(self.lib.pmx_qualhisto(self.ctx, opt, C.byref(st)), "pmx_qualhisto")
        return self._qdict(st)

    def qualhisto_device(self, dev_ptr: int, opt: int = N.INQUA, use_stored: bool = False):
        self._chk(self.lib.pmx_qualhisto_device(self.ctx, opt, int(use_stored), C.c_void_p(dev_ptr)),
                  "pmx_qualhisto_device")

    @staticmethod
    def _par(par: dict | None):
        if par is None:
            return None, []
        a = np.ascontiguousarray(par["a"], np.int32)
        b = np.ascontiguousarray(par["b"], np.int32)
        o = np.ascontiguousarray(par["owner"], np.int32)
        pe = N.ParEdges()
        pe.n, pe.a, pe.b, pe.owner = len(a), _ip(a), _ip(b), _ip(o)
        pe.myrank, pe.exact_once = int(par.get("myrank", 0)), int(par.get("exact_once", 0))
        keep = [a, b, o, pe]
        if par.get("tag") is not None:
            t = np.ascontiguousarray(par["tag"], np.uint16)
            pe.tag = t.ctypes.data_as(N.u16ptr)
            keep.append(t)
        return C.byref(pe), keep

    def upload_surface(self, surface: dict | None):
        """Mmg's surface data of the uploaded group (pmx_upload_surface):
        {"xt" (ne+1,) tetra[k].xt, "xtag" (nxt+1, 6) xtetra[x].tag, "n" (np+1, 3)
        point[i].n, "xp" (np+1,) point[i].xp, "n1"/"n2" (nxp+1, 3) xpoint[x].n1/n2};
        None: no surface data (no xTetra, zero normals)."""
        if surface is None:
            self._chk(self.lib.pmx_upload_surface(self.ctx, None), "pmx_upload_surface")
            return
        xt = np.ascontiguousarray(surface["xt"], np.int32)
        xtag = np.ascontiguousarray(surface["xtag"], np.uint16).reshape(-1, 6)
        n = np.ascontiguousarray(surface["n"], np.float64).reshape(-1, 3)
        xp = np.ascontiguousarray(surface["xp"], np.int32)
        n1 = np.ascontiguousarray(surface["n1"], np.float64).reshape(-1, 3)
        n2 = np.ascontiguousarray(surface["n2"], np.float64).reshape(-1, 3)
        sv = N.SurfaceView()
        sv.nxt, sv.nxp = xtag.shape[0] - 1, n1.shape[0] - 1
        sv.tetra_xt, sv.tetra_stride = _ip(xt), 4
        sv.xtetra_tag, sv.xtetra_stride = xtag.ctypes.data_as(N.u16ptr), 12
        sv.point_n, sv.point_xp, sv.point_stride = _dp(n), _ip(xp), 24
        # point_n / point_xp share one stride in the ABI (MMG5_Point): pack them
        rec = np.zeros(n.shape[0], dtype=[("n", np.float64, 3), ("xp", np.int32), ("pad", np.int32)])
        rec["n"], rec["xp"] = n, xp
        sv.point_n = C.cast(C.c_void_p(rec.ctypes.data), N.dptr)
        sv.point_xp = C.cast(C.c_void_p(rec.ctypes.data + 24), N.iptr)
        sv.point_stride = rec.dtype.itemsize
        sv.xpoint_n1, sv.xpoint_n2, sv.xpoint_stride = _dp(n1), _dp(n2), 24
        self._chk(self.lib.pmx_upload_surface(self.ctx, C.byref(sv)), "pmx_upload_surface")

    def prilen(self, met_rid_typ: int = 0, par: dict | None = None) -> dict:
        """par: {"a", "b", "owner", "myrank", "exact_once"} (distributed PMMG_prilen)."""
        st = N.LenStats()
        pp, keep = self._par(par)
        self._chk(self.lib.pmx_prilen(self.ctx, met_rid_typ, pp, C.byref(st)), "pmx_prilen")
        del keep
        return self._ldict(st)

    def prilen_device(self, dev_ptr: int, met_rid_typ: int = 0, par: dict | None = None):
        pp, keep = self._par(par)
        self._chk(self.lib.pmx_prilen_device(self.ctx, met_rid_typ, pp, C.c_void_p(dev_ptr)),
                  "pmx_prilen_device")
        del keep

    def upload_new_tets(self, tets: np.ndarray):
        """The new mesh's tets, (ne+1, 4) with 0-based point indices (v[0] < 0:
        deleted), for pmx_promote_background / pmx_new_mesh_qual."""
        tv = _tets_1based(tets)
        self._chk(self.lib.pmx_upload_new_tets(self.ctx, _ip(tv), 16, tv.shape[0] - 1),
                  "pmx_upload_new_tets")
        self.n_new_tets = tv.shape[0] - 1

    def promote_background(self, new_mesh: Mesh, sols: list[np.ndarray] | None = None,
                           adja: bool = True):
        """The last step's new points + results become the background (device
        resident).  new_mesh: the new mesh (its trias/adjt/hausd and, with
        adja=True, its adjacency are read; coordinates and tets are not);
        sols: the (n, size) result arrays of the last download (values of the
        rows the step did not write)."""
        mv = mesh_view(new_mesh)
        if not adja:
            mv.adja = None
        arr = [np.ascontiguousarray(s, np.float64) for s in (sols or [])]
        views = (N.SolView * max(len(arr), 1))()
        for i, a in enumerate(arr):
            views[i].size = a.shape[1] if a.ndim == 2 else 1
            views[i].m = _dp(a)                 # pmx_download's layout: entry 0 = point 1
        self._chk(self.lib.pmx_promote_background(self.ctx, C.byref(mv), len(arr), views),
                  "pmx_promote_background")
        self.npts = 0

    def new_mesh_qual(self, tets: np.ndarray | None, opt: int = N.INQUA, dev_ptr: int = 0,
                      met_rid_typ: int = 0) -> np.ndarray:
        """PMMG_tetraQual on the new mesh after the last step: tets (ne+1, 4)
        with indices of the uploaded points (0-based here, v[0] < 0: deleted);
        None: the tets of the last upload_new_tets."""
        tv = _tets_1based(tets) if tets is not None else None
        q = np.zeros((tv.shape[0] if tv is not None else self.n_new_tets + 1))
        self._chk(self.lib.pmx_new_mesh_qual(self.ctx, _ip(tv), 16, tv.shape[0] - 1 if tv is not None else 0,
                                             opt, met_rid_typ, _dp(q), len(q), C.c_void_p(dev_ptr or None)),
                  "pmx_new_mesh_qual")
        if tv is not None:
            self.n_new_tets = tv.shape[0] - 1
        return q

    def new_mesh_qual_synced(self, met: np.ndarray | None, opt: int = N.INQUA, met_rid_typ: int = 1,
                             out: np.ndarray | None = None) -> np.ndarray:
        """PMMG_tetraQual after the interpolation on the caller's metric
        (Mmg layout, (np+1, size), entry 0 unused; None: no metric), the new
        tets being the last points view's.  out: None -> a dense (ne+1,) array;
        a structured array with a "qual" field (MMG_TETRA records) -> written
        in place for the valid tets only (pmx_new_mesh_qual_synced, strided)."""
        mv = None
        if met is not None:
            met = np.ascontiguousarray(met, np.float64)
            mv = N.SolView()
            mv.size, mv.m = met.shape[1], _dp(met)
        if out is None:
            q = np.zeros(self.n_new_tets + 1)
            ptr, stride = _dp(q), 8
        else:
            if (out.ndim != 1 or not out.flags.c_contiguous or out.dtype.fields is None or "qual" not in
                    out.dtype.fields or out.dtype.fields["qual"][0] != np.float64 or
                    out.shape[0] < self.n_new_tets + 1):
                raise ValueError("out: a contiguous 1-D record array with a float64 'qual' field, "
                                 "one record per new tet plus slot 0")
            q = out
            base = out.ctypes.data + out.dtype.fields["qual"][1]
            ptr, stride = C.cast(C.c_void_p(base), N.dptr), out.dtype.itemsize
        self._chk(self.lib.pmx_new_mesh_qual_synced(self.ctx, C.byref(mv) if mv is not None else None, opt,
                                                    met_rid_typ, ptr, stride, q.shape[0], None),
                  "pmx_new_mesh_qual_synced")
        return q

    def comm_init(self, nranks: int, uid: bytes, rank: int) -> int:
        c = C.c_void_p()
        self._chk(self.lib.pmx_comm_init(self.ctx, C.byref(c), nranks, uid, rank), "pmx_comm_init")
        return c.value

    @staticmethod
    def comm_destroy(comm: int):
        if comm and not N.load().pmx_comm_destroy(C.c_void_p(comm)):
            raise RuntimeError("pmx_comm_destroy failed")

    def qualhisto_allreduce(self, comm: int, nranks: int, dev_ptr: int, ngrp: int = 1) -> dict:
        st = N.QualStats()
        self._chk(self.lib.pmx_qualhisto_allreduce(self.ctx, C.c_void_p(comm), nranks,
                                                   C.c_void_p(dev_ptr), ngrp, C.byref(st)),
                  "pmx_qualhisto_allreduce")
        return self._qdict(st)

    def prilen_allreduce(self, comm: int, nranks: int, dev_ptr: int) -> dict:
        st = N.LenStats()
        self._chk(self.lib.pmx_prilen_allreduce(self.ctx, C.c_void_p(comm), nranks, C.c_void_p(dev_ptr),
                                                C.byref(st)), "pmx_prilen_allreduce")
        return self._ldict(st)


def comm_unique_id() -> bytes:
    lib = N.load()
    buf = C.create_string_buffer(256)
    n = lib.pmx_comm_unique_id(buf, 256)
    if not n:
        raise RuntimeError("pmx_comm_unique_id failed")
    return buf.raw[:n]
