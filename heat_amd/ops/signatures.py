"""ctypes signatures of native kernels beyond the core set (registered when present)."""
import ctypes

c_void_p, c_int, c_int64, c_uint64, c_float, c_double = (ctypes.c_void_p, ctypes.c_int, ctypes.c_int64,
                                                         ctypes.c_uint64, ctypes.c_float, ctypes.c_double)

SIGNATURES = {
    "ha_h3_topk": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int, c_int64, c_void_p, c_int, c_int,
                           c_void_p, c_void_p, c_void_p]),
    "ha_h3_topk_chunks": (c_int, [c_int, c_int]),
    "ha_split_absmax": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p]),
    "ha_split3": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                          c_void_p, c_int64, c_void_p, c_void_p]),
    "ha_split3_rows": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p, c_void_p, c_void_p]),
    "ha_split_unscale": (c_int, [c_void_p, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_void_p]),
    "ha_cdist": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int, c_int64, c_int64, c_void_p, c_int64, c_int,
                         c_float, c_void_p]),
    "ha_threefry_fill": (c_int, [c_void_p, c_int64, c_int64, c_uint64, c_uint64, c_uint64, c_int, c_int, c_double,
                                 c_double, c_void_p]),
    "ha_lasso_pass": (c_int, [c_void_p, c_int64, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                              c_void_p]),
    "ha_h3_fpad": (c_int, [c_int]),
    "ha_h3_pack_points": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p]),
    "ha_h3_workspace_bytes": (c_int64, [c_int, c_int]),
    "ha_h3_assign": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int, c_int64, c_void_p, c_void_p,
                             c_void_p, c_void_p]),
    "ha_h3_assign_certified": (c_int, [c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int, c_int64, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_void_p]),
    "ha_cdist_h3_fpad": (c_int, [c_int]),
    "ha_cdist_h3_rows": (c_int64, [c_int64]),
    "ha_cdist_h3_pack": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_void_p]),
    "ha_cdist_h3": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_int64, c_int,
                            c_float, c_void_p]),
    "ha_lasso_prepare": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p]),
    "ha_lasso_update": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_float, c_float, c_void_p, c_int, c_void_p]),
}
