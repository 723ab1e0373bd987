"""ctypes binding of ``libpmx_transfer.so`` (the C ABI in include/pmx_transfer.h).

Loading fails loudly: there is no Python or CPU fallback for the transfer path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpmx_transfer.so")

i64 = C.c_int64
dptr = C.POINTER(C.c_double)
iptr = C.POINTER(C.c_int)
u16ptr = C.POINTER(C.c_uint16)


class MeshView(C.Structure):
    _fields_ = [
        ("np", i64), ("ne", i64), ("nt", i64),
        ("point_c", dptr), ("point_stride", i64),
        ("tetra_v", iptr), ("tetra_stride", i64),
        ("adja", iptr),
        ("tria_v", iptr), ("tria_stride", i64),
        ("adjt", iptr),
        ("hausd", C.c_double),
    ]


class SolView(C.Structure):
    _fields_ = [("size", C.c_int), ("m", dptr)]


class PointsView(C.Structure):
    _fields_ = [
        ("first", i64), ("last", i64),
        ("c", dptr), ("stride", i64),
        ("tag", u16ptr), ("tag_stride", i64),
        ("tetra_v", iptr), ("tetra_stride", i64), ("ne", i64),
    ]


class LocateStats(C.Structure):
    _fields_ = [
        ("nvol", i64), ("nbdy", i64), ("nexhaust", i64), ("nclosest", i64),
        ("stepmin", i64), ("stepmax", i64), ("stepav", C.c_double),
    ]


class WaveStats(C.Structure):
    _fields_ = [("waves", i64), ("located", i64), ("step_sum", i64), ("lane_steps", i64),
                ("wave_max_hist", i64 * 16)]


class RunOpts(C.Structure):
    _fields_ = [
        ("hint_stride", C.c_int), ("max_walk", C.c_int),
        ("hsiz", C.c_double), ("timing", C.c_int), ("flags", C.c_int),
    ]


# pmx_run_opts.flags (include/pmx_transfer.h)
RUN_REFERENCE_WALK = 0x1
RUN_NO_INLINE_TIES = 0x2
RUN_RECORD_STARTS = 0x4
RUN_SERIAL_SURFACE = 0x8
RUN_FRESH_BACKGROUND = 0x10
RUN_DEBUG_BARRIER_TIMEOUT = 0x100
RUN_EAGER_DOWNLOAD = 0x20
RUN_SEQUENTIAL_SURFACE = 0x40
RUN_SEQUENTIAL_VOLUME = 0x80


class Group(C.Structure):
    _fields_ = [
        ("mesh", MeshView), ("points", PointsView),
        ("met", C.POINTER(SolView)), ("fields", C.POINTER(SolView)), ("nsols", C.c_int),
        ("hsiz", C.c_double),
        ("old_mesh", MeshView), ("old_met", C.POINTER(SolView)), ("old_fields", C.POINTER(SolView)),
    ]


class QualStats(C.Structure):
    _fields_ = [
        ("ne", i64), ("np", i64), ("max", C.c_double), ("min", C.c_double), ("avg", C.c_double),
        ("iel", i64), ("good", i64), ("med", i64), ("his", i64 * 5), ("nrid", i64),
        ("iel_grp", C.c_int), ("cpu", C.c_int),
    ]


class LenStats(C.Structure):
    _fields_ = [
        ("ned", i64), ("nullEdge", i64), ("avlen", C.c_double), ("lmin", C.c_double),
        ("lmax", C.c_double), ("amin", i64), ("bmin", i64), ("amax", i64), ("bmax", i64),
        ("hl", i64 * 9), ("cpu_min", C.c_int), ("cpu_max", C.c_int),
    ]


class QualPart(C.Structure):
    """pmx_qual_part: the device partial of one group (15 x 8 B)."""
    _fields_ = [
        ("avg", C.c_double), ("max", C.c_double), ("min", C.c_double),
        ("iel", i64), ("ne", i64), ("np", i64), ("good", i64), ("med", i64), ("nrid", i64),
        ("his", i64 * 5), ("iel_grp", i64),
    ]


class LenPart(C.Structure):
    """pmx_len_part: the device partial of one group (18 x 8 B)."""
    _fields_ = [
        ("avlen", C.c_double), ("lmin", C.c_double), ("lmax", C.c_double),
        ("amin", i64), ("bmin", i64), ("amax", i64), ("bmax", i64), ("ned", i64),
        ("nullEdge", i64), ("hl", i64 * 9),
    ]


class ParEdges(C.Structure):
    _fields_ = [
        ("n", i64), ("a", iptr), ("b", iptr), ("owner", iptr), ("myrank", C.c_int),
        ("exact_once", C.c_int), ("tag", u16ptr),
    ]


class SurfaceView(C.Structure):
    """pmx_surface_view: Mmg's surface data through strides."""
    _fields_ = [
        ("nxt", i64), ("nxp", i64),
        ("tetra_xt", iptr), ("tetra_stride", i64),
        ("xtetra_tag", u16ptr), ("xtetra_stride", i64),
        ("point_n", dptr), ("point_xp", iptr), ("point_stride", i64),
        ("xpoint_n1", dptr), ("xpoint_n2", dptr), ("xpoint_stride", i64),
    ]


INQUA, OUTQUA, LESQUA = 0, 1, 2


class MeditInfo(C.Structure):
    _fields_ = [("np", i64), ("ne", i64), ("nt", i64), ("nreq", i64), ("dim", C.c_int),
                ("version", C.c_int)]


# symbol -> (restype, argtypes); every function declared in include/pmx_transfer.h
SIGNATURES = {
    "pmx_create": (C.c_void_p, [C.c_int]),
    "pmx_destroy": (None, [C.c_void_p]),
    "pmx_last_error": (C.c_char_p, [C.c_void_p]),
    "pmx_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pmx_synchronize": (C.c_int, [C.c_void_p]),
    "pmx_device_info": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "pmx_upload_background": (C.c_int, [C.c_void_p, C.POINTER(MeshView), C.c_int, C.POINTER(SolView), C.c_int]),
    "pmx_upload_points": (C.c_int, [C.c_void_p, C.POINTER(PointsView)]),
    "pmx_run": (C.c_int, [C.c_void_p, C.POINTER(RunOpts)]),
    "pmx_download": (C.c_int, [C.c_void_p, C.POINTER(SolView), i64, iptr, iptr, iptr]),
    "pmx_download_starts": (C.c_int, [C.c_void_p, iptr, i64]),
    "pmx_download_border": (C.c_int, [C.c_void_p, iptr, iptr, i64]),
    "pmx_step_ready": (C.c_int, [C.c_void_p]),
    "pmx_locate_stats_get": (C.c_int, [C.c_void_p, C.POINTER(LocateStats)]),
    "pmx_locate_wave_stats": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(WaveStats)]),
    "pmx_seq_surface_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "pmx_seq_volume_stats": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "pmx_device_buffer": (C.c_void_p, [C.c_void_p, C.c_int]),
    "pmx_device_alloc": (C.c_void_p, [C.c_void_p, C.c_size_t]),
    "pmx_device_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pmx_device_download": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "pmx_device_upload": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "pmx_debug_hint_grid": (C.c_int64, [C.c_void_p, C.c_void_p, C.c_int64]),
    "pmx_build_adja": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                 C.c_void_p]),
    "pmx_build_bdry": (C.c_int64, [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_int64,
                                   C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]),
    "pmx_topo_ms": (C.c_double, [C.c_void_p]),
    "pmx_kernel_ms": (C.c_double, [C.c_void_p, C.c_int]),
    "pmx_timing_reset": (C.c_int, [C.c_void_p]),
    "PMX_interpMetricsAndFields": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(Group), iptr, C.c_int]),
    "PMX_interpMetricsAndFields_groups": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(Group), iptr,
                                                    C.c_int]),
    "PMX_copyMetricsAndFields_point": (C.c_int, [C.c_void_p, C.POINTER(Group), u16ptr, i64, iptr, C.c_int, C.c_int]),
    "pmx_tetra_qual": (C.c_int, [C.c_void_p, C.c_int, dptr, i64]),
    "pmx_upload_point_tags": (C.c_int, [C.c_void_p, u16ptr, i64]),
    "pmx_upload_surface": (C.c_int, [C.c_void_p, C.POINTER(SurfaceView)]),
    "pmx_count_nodes": (C.c_int, [C.c_void_p, iptr, iptr, i64, iptr, i64, C.c_int, C.POINTER(i64)]),
    "pmx_qualhisto_device": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_void_p]),
    "pmx_qualhisto": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(QualStats)]),
    "pmx_prilen_device": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(ParEdges), C.c_void_p]),
    "pmx_prilen": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(ParEdges), C.POINTER(LenStats)]),
    "pmx_new_mesh_qual": (C.c_int, [C.c_void_p, iptr, i64, i64, C.c_int, C.c_int, dptr, i64, C.c_void_p]),
    "pmx_new_mesh_qual_synced": (C.c_int, [C.c_void_p, C.POINTER(SolView), C.c_int, C.c_int, dptr, i64,
                                          i64, C.c_void_p]),
    "pmx_upload_new_tets": (C.c_int, [C.c_void_p, iptr, i64, i64]),
    "pmx_set_residency": (C.c_int, [C.c_void_p, C.c_int]),
    "pmx_copy_required": (C.c_int, [C.c_void_p, iptr, C.c_int]),
    "pmx_promote_background": (C.c_int, [C.c_void_p, C.POINTER(MeshView), C.c_int, C.POINTER(SolView)]),
    "pmx_qual_fold": (C.c_int, [C.POINTER(QualPart), iptr, C.c_int, C.POINTER(QualStats)]),
    "pmx_len_fold": (C.c_int, [C.POINTER(LenPart), C.c_int, C.POINTER(LenStats)]),
    "pmx_comm_unique_id": (C.c_int, [C.c_char_p, C.c_int]),
    "pmx_comm_init": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_char_p, C.c_int]),
    "pmx_comm_destroy": (C.c_int, [C.c_void_p]),
    "pmx_qualhisto_allreduce": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                                          C.POINTER(QualStats)]),
    "pmx_prilen_allreduce": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.POINTER(LenStats)]),
    "pmx_medit_last_error": (C.c_char_p, []),
    "pmx_medit_mesh_info": (C.c_int, [C.c_char_p, C.POINTER(MeditInfo)]),
    "pmx_medit_mesh_read": (C.c_int, [C.c_char_p, C.POINTER(MeditInfo), dptr, iptr, iptr, iptr, iptr, iptr, iptr]),
    "pmx_medit_mesh_write": (C.c_int, [C.c_char_p, i64, dptr, iptr, i64, iptr, iptr, i64, iptr, iptr,
                                       i64, iptr]),
    "pmx_medit_sol_info": (C.c_int, [C.c_char_p, C.POINTER(i64), C.POINTER(C.c_int), iptr]),
    "pmx_medit_sol_read": (C.c_int, [C.c_char_p, i64, C.c_int, iptr, C.POINTER(dptr)]),
    "pmx_medit_sol_write": (C.c_int, [C.c_char_p, i64, C.c_int, iptr, C.POINTER(dptr)]),
}

_lib = None


def load() -> C.CDLL:
    """Load the HIP extension; raise if it is missing (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python -m parmmg_amd.build` "
            "(the transfer path has no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib
