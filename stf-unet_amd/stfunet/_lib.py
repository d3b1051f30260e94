"""ctypes binding of the gfx950 C-ABI libraries (include/stfunet.h).

The sources are built in-tree by ``make -C stf-unet_amd/csrc`` (or
``__graft_entry__.build()``) twice: ``stfunet/libstfunet_hip.so`` (bf16 activation
storage, the default) and ``stfunet/libstfunet_hip_f16.so`` (fp16 storage: the
reference's ``autocast(float16)`` + GradScaler numerics).  Same entry points; the
launches go to the library of the *active storage dtype* (``storage(dtype)``, set by
the models around their forward / backward).  There is no fallback: if a library is
missing or fails to load, every op raises.  ``torch`` is imported first so the HIP
runtime torch ships (soname ``libamdhip64.so.7``) is the one the libraries bind to --
one runtime per process.
"""
import contextlib
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libstfunet_hip.so")
# A/B measurements: STF_LIB / STF_LIB_F16 point at other builds of the same libraries
# (tools/ab_lib.sh); STF_LIB alone also moves the fp16 build to its directory
LIB_PATH = os.environ.get("STF_LIB", LIB_PATH)
LIB_PATH_F16 = os.environ.get("STF_LIB_F16", os.path.join(os.path.dirname(LIB_PATH), "libstfunet_hip_f16.so"))
LIB_PATHS = {torch.bfloat16: LIB_PATH, torch.float16: LIB_PATH_F16}
STORAGE_CODE = {torch.bfloat16: 0, torch.float16: 1}     # stf_storage_type()

BUILD_INFO = os.path.join(_HERE, "build_info.json")     # written by __graft_entry__.build()
_SRC_DIRS = (os.path.join(_HERE, "..", "csrc"), os.path.join(_HERE, "..", "..", "include"))


def _sha(paths):
    import hashlib
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def source_digest():
    """sha256 prefix over the HIP sources, their headers and the Makefile (None if absent)."""
    files = []
    for d in _SRC_DIRS:
        if os.path.isdir(d):
            files += sorted(os.path.join(d, f) for f in os.listdir(d)
                            if f.endswith((".hip", ".h")) or f == "Makefile")
    return _sha(files) if files else None


def build_info():
    """Which build is loaded: digests of the two libraries as they are on disk, the source digest
    recorded when they were built (build_info.json) and the digest of the sources present now --
    src_recorded == src_now says the libraries were built from these sources."""
    import json
    info = {"lib": {}, "src_recorded": None, "src_now": source_digest()}
    for dt, path in LIB_PATHS.items():
        key = "bf16" if dt == torch.bfloat16 else "fp16"
        info["lib"][key] = _sha([path]) if os.path.exists(path) else None
    try:
        with open(BUILD_INFO) as f:
            rec = json.load(f)
        info["src_recorded"] = rec.get("src")
        info["lib_recorded"] = rec.get("lib")
    except (OSError, ValueError):
        pass
    info["current"] = (info["src_recorded"] is not None and info["src_recorded"] == info["src_now"]
                       and info.get("lib_recorded") == info["lib"])
    return info


c_uint = ctypes.c_uint
c_int, c_void_p, c_float, c_size_t, c_int64 = (ctypes.c_int, ctypes.c_void_p, ctypes.c_float,
                                                ctypes.c_size_t, ctypes.c_int64)
P = c_void_p


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("N", "Hs", "Ws", "Cs", "src_cstride", "Hd", "Wd", "R", "S",
                                     "stride", "pad", "transposed")]


class LstmEpi(ctypes.Structure):
    _fields_ = [("c_prev", P), ("c_out", P), ("h_out", P), ("h_cstride", c_int), ("gates", P),
                ("backward", c_int), ("dh", P), ("dh_cstride", c_int), ("dc_next", P), ("dc_prev", P),
                ("dgates", P)]


class BnrEpi(ctypes.Structure):
    _fields_ = [("y", P), ("y_cstride", c_int), ("scale", P), ("shift", P), ("mean", P), ("invstd", P),
                ("relu", c_int), ("partial", P)]


class IgemmArgs(ctypes.Structure):
    _fields_ = [("g", ConvGeom), ("src", P), ("wgt", P), ("Nout", c_int), ("dst", P),
                ("dst_cstride", c_int), ("bias", P), ("stats", P), ("scatter2x2", c_int),
                ("group_rows", c_int), ("accumulate", c_int), ("lstm", ctypes.POINTER(LstmEpi)),
                ("bnr", ctypes.POINTER(BnrEpi)), ("ws", P)]


class WgradArgs(ctypes.Structure):
    _fields_ = [("g", ConvGeom), ("dy", P), ("dy_cstride", c_int), ("Nout", c_int), ("x", P),
                ("ws", P), ("splits", c_int), ("grid_blocks", c_int)]


# name -> (restype, argtypes)
_SIGS = {
    "stf_igemm_stat_tiles": (c_int, [ctypes.POINTER(IgemmArgs)]),
    "stf_igemm_ws_bytes": (c_size_t, [ctypes.POINTER(IgemmArgs)]),
    "stf_igemm_bnr_tiles": (c_int, [ctypes.POINTER(IgemmArgs)]),
    "stf_igemm_kernel_name": (ctypes.c_char_p, [ctypes.POINTER(IgemmArgs)]),
    "stf_wgrad_kernel_name": (ctypes.c_char_p, [ctypes.POINTER(WgradArgs)]),
    "stf_igemm": (c_int, [ctypes.POINTER(IgemmArgs), P]),
    "stf_wgrad_plan": (c_int, [ctypes.POINTER(WgradArgs), ctypes.POINTER(c_int), ctypes.POINTER(c_size_t)]),
    "stf_wgrad": (c_int, [ctypes.POINTER(WgradArgs), P]),
    "stf_wgrad_reduce": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "stf_channel_sum": (c_int, [P, c_int, c_int, c_int, P, P, P]),
    "stf_bn_finalize": (c_int, [P, c_int, c_int, c_int, c_int64, P, P, c_float, c_float, P, P, P, P, P, P, P]),
    "stf_bn_running_batch": (c_int, [P, c_int, P]),
    "stf_bn_groupsum_batch": (c_int, [P, c_int, P]),
    "stf_bn_act": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, c_int, P, P, P, c_int, P,
                           P]),
    "stf_bn_bwd_tiles": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "stf_bn_bwd_reduce": (c_int, [P, c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, P, c_int, P,
                                  c_int, P, P, P]),
    "stf_bn_bwd_finalize": (c_int, [P, c_int, c_int, c_int, c_int64, P, P, P, P, P, P, P]),
    "stf_bn_bwd_apply_tiles": (c_int, [c_int64, c_int]),
    "stf_bn_bwd_apply": (c_int, [P, c_int, P, c_int, c_int64, c_int, c_int, P, P, P, P, c_int, P, P, P]),
    "stf_head_fwd": (c_int, [P, c_int, c_int, c_int, c_int, P, P, P, P, c_int, P, P]),
    "stf_head_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P, P, P, c_int, P, P, P, P, P, P]),
    "stf_head_tiles": (c_int, [c_int, c_int, c_int, c_int]),
    "stf_loss_scratch_floats": (c_int, [c_int, c_int]),
    "stf_loss_fwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P]),
    "stf_loss_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P, P]),
    "stf_adamw": (c_int, [P, P, P, P, c_int64, c_float, c_float, c_float, c_float, c_float, c_float, c_float,
                          P]),
    "stf_adamw_dev": (c_int, [P, P, P, P, c_int64, P, c_float, c_float, c_float, c_float, P]),
    "stf_adamw_amp": (c_int, [P, P, P, P, c_int64, P, P, P, c_float, c_float, c_float, c_float, P]),
    "stf_pack_input": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "stf_pack_weight": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "stf_pack_weights": (c_int, [P, c_int, c_int64, P]),
    "stf_augment_frames": (c_int, [P, P, c_int, P, P, c_int, c_int, c_float, c_float, P, P]),
    "stf_augment_masks": (c_int, [P, P, c_int, P, c_int, P, P]),
    "stf_pack_tiles": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int]),
    "stf_pack_weights_tiled": (c_int, [P, c_int, c_int, P]),
    "stf_pack_sequence": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "stf_eval_counts": (c_int, [P, P, c_int, c_int, c_int64, c_int64, P, P, P]),
    "stf_lstm_coop_sync_bytes": (c_size_t, [c_int, c_int]),
    "stf_lstm_coop_supported": (c_int, [c_int]),
    "stf_lstm_coop_fwd": (c_int, [P, P, P, c_int, c_int, c_int, P, P, c_int, P, P, c_int, c_uint, P]),
    "stf_lstm_coop_bwd": (c_int, [P, P, P, c_int, c_int, c_int, P, c_int, P, P, c_int, P, c_int, c_uint, P]),
    "stf_lstm_coop_error": (c_int, [P, c_int, c_int, P, P]),
    "stf_bilinear_ac_fwd": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, P]),
    "stf_bilinear_ac_bwd": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, P]),
    "stf_stat_sums": (c_int, [P, c_int, c_int, c_int, c_int, P, P]),
    "stf_bilinear_ac_bwd_tsum": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int64, c_int64, c_int,
                                         c_int, P]),
    "stf_eval_counts_sm": (c_int, [P, P, P, c_int, c_int, c_int64, c_int64, P, P, P]),
    "stf_tofts_forward": (c_int, [P, P, P, c_int, c_int, P, P, P, P, P, c_int, c_float, P, P]),
    "stf_tofts_fit": (c_int, [P, c_int, c_int, P, P, P, P, P, c_int, c_float, c_int, c_int, P, c_float, c_float,
                              c_float, P, P, P]),
    "stf_stem_im2col": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P,
                                P]),
    "stf_stem_conv7_grid": (c_int, [c_int, c_int, c_int, c_int]),
    "stf_stem_conv7": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, P, P]),
    "stf_stem_wgrad7": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "stf_stem_dgrad7": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "stf_maxpool3s2_fwd": (c_int, [P, c_int, c_int, c_int, c_int, P, P, P]),
    "stf_maxpool3s2_bwd": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P]),
    "stf_bn_act_maxpool3s2": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "stf_bn_bwd_reduce_pool3": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P, P]),
    "stf_bn_bwd_apply_pool3": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "stf_lstm_pack": (c_int, [P, P, P, P, c_int, P, P, P, P]),
    "stf_lstm_unpack_grad": (c_int, [P, P, c_int, P, P, P, P, P]),
    "stf_lstm_seq_fwd": (c_int, [P, P, P, c_int, c_int, c_int, P, P, c_int, P]),
    "stf_lstm_seq_supported": (c_int, [c_int]),
    "stf_lstm_seq_bwd": (c_int, [P, P, P, P, c_int, c_int, c_int, P, P, c_int, P, P, c_int, P]),
    "stf_lstm_cell_bwd": (c_int, [P, P, P, P, c_int, P, P, P, c_int64, c_int, P]),
    "stf_pk_resize": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P]),
    "stf_plan_create": (c_void_p, []),
    "stf_plan_destroy": (None, [P]),
    "stf_plan_record": (c_int, [P]),
    "stf_plan_stop": (c_int, []),
    "stf_plan_size": (c_int, [P]),
    "stf_plan_tag": (c_int, [ctypes.c_char_p, ctypes.c_double]),
    "stf_plan_tag_end": (c_int, []),
    "stf_plan_replay": (c_int, [P, c_int, c_int, ctypes.c_char_p]),
    "stf_plan_timing": (c_int, [P, ctypes.POINTER(c_int), ctypes.POINTER(ctypes.c_double),
                                ctypes.POINTER(ctypes.c_double)]),
    "stf_stream_wait": (c_int, [P, P]),
    "stf_memset": (c_int, [P, c_int, c_size_t, P]),
    "stf_copy_rows": (c_int, [P, c_int64, P, c_int64, c_int, c_int, P]),
    "stf_i64_add_batch": (c_int, [ctypes.POINTER(c_void_p), c_int, c_int64, P]),
    "stf_error_string": (ctypes.c_char_p, [c_int]),
    "stf_abi_version": (c_int, []),
    "stf_storage_type": (c_int, []),
}

EXPORTED = tuple(_SIGS)
_libs = {}
_active = torch.bfloat16          # storage dtype of the launches issued now
_FNS = {}                         # dtype -> {entry point name -> bound function}
_FN = _FNS.setdefault(_active, {})


def load(dtype=None):
    """Load (once) and return the CDLL of ``dtype``'s storage (default: the active
    one); raises RuntimeError if unavailable or built for another storage type."""
    dtype = _active if dtype is None else dtype
    lib = _libs.get(dtype)
    if lib is not None:
        return lib
    if dtype not in LIB_PATHS:
        raise ValueError(f"no stfunet library for storage dtype {dtype} (bf16 or fp16)")
    path = LIB_PATHS[dtype]
    if not os.path.exists(path):
        raise RuntimeError(f"stfunet HIP library not built ({path}); run `make -C stf-unet_amd/csrc` "
                           "or __graft_entry__.build()")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.stf_storage_type() != STORAGE_CODE[dtype]:
        raise RuntimeError(f"{path} was built for another storage type ({lib.stf_storage_type()})")
    _libs[dtype] = lib
    return lib


def storage_dtype():
    """The 16-bit activation storage dtype the launches issued now use."""
    return _active


def storage_for(requested=None):
    """The storage a model runs with: ``requested`` (a model's ``storage_dtype``) if set,
    else fp16 inside ``torch.autocast('cuda', dtype=torch.float16)`` -- the reference's
    ``--amp`` path (train_and_eval.py:389, autocast's cuda default dtype) -- else bf16."""
    if requested is not None:
        return requested
    if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.float16:
        return torch.float16
    return torch.bfloat16


@contextlib.contextmanager
def storage(dtype):
    """Route launches to the bf16 or the fp16 library inside the block.  The models
    enter it around their forward and backward (one model's forward and backward
    never overlap in time; two models of different storage must not run
    concurrently)."""
    global _active, _FN
    if dtype not in LIB_PATHS:
        raise ValueError(f"activation storage must be torch.bfloat16 or torch.float16, not {dtype}")
    prev = _active
    _active, _FN = dtype, _FNS.setdefault(dtype, {})
    try:
        yield
    finally:
        _active, _FN = prev, _FNS.setdefault(prev, {})


class HipError(RuntimeError):
    pass


def check(rc, what=""):
    if rc != 0:
        msg = load().stf_error_string(rc).decode()
        raise HipError(f"{what}: {msg} (code {rc})")


_FN = {}


def call(name, *args):
    f = _FN.get(name)
    if f is None:
        f = _FN[name] = getattr(load(_active), name)
    rc = f(*args)
    if rc != 0:
        check(rc, name)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


_get_device = torch._C._cuda_getDevice


def stream():
    """Raw hipStream_t of torch's current stream on the current device, as a plain int
    (every entry point declares its stream argument c_void_p, which ctypes fills from an
    int; the raw accessor skips torch.cuda.current_stream()'s Python wrapper: ~9 us ->
    <1 us per launch, and the STF step is host-bound with ~600 launches from Python)."""
    if _raw_stream is not None:
        return _raw_stream(_get_device())
    return torch.cuda.current_stream().cuda_stream
