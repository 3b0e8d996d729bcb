"""ctypes binding of libsatmi.so (include/satmi.h).

The library is built in-tree (`make -C sat-mpi-stana-andrei_amd`, or
`__graft_entry__.build()`).  There is no CPU fallback: if the library or a GPU
is missing, every solver call raises SatmiError.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, os.environ.get("SATMI_LIB_VARIANT", "libsatmi.so"))   # A/B builds: libsatmi_*.so

# include/satmi.h constants
OK = 0
MODE_REF = 0
MODE_SOUND = 1
NCOUNTERS = 8
COUNTER_NAMES = ("nodes", "decisions", "unit_props", "pure_assigns", "conflicts", "solutions", "rounds",
                 "ticks")
DPLL_EXHAUSTED, DPLL_STOPPED, DPLL_NODE_LIMIT, DPLL_TIMEOUT, DPLL_TOO_LARGE = range(5)
STATUS_NAMES = {0: "exhausted", 1: "stopped", 2: "node_limit", 3: "timeout", 4: "too_large"}
RES_SAT, RES_UNSAT, RES_LIMIT = 1, 0, -1
KERNEL_AUTO, KERNEL_GENERAL, KERNEL_SCAN, KERNEL_INC, KERNEL_WIDE = 0, 1, 2, 3, 4

# exported symbols, checked by tests/test_capi_symbols.py against include/satmi.h
EXPORTED = (
    "satmi_abi_version", "satmi_last_error", "satmi_device_count", "satmi_set_device", "satmi_synchronize",
    "satmi_malloc", "satmi_free", "satmi_memcpy_h2d", "satmi_memcpy_d2h", "satmi_stream_synchronize",
    "satmi_dpll_batch_device", "satmi_dpll_batch_host", "satmi_dpll_lds_bytes", "satmi_resolution_host",
    "satmi_dp_host", "satmi_dpll_scan_lds_bytes", "satmi_dpll_set_kernel", "satmi_dpll_plan",
    "satmi_dpll_launch_span", "satmi_wallclock_hz", "satmi_resolution_debug_slot_base",
    "satmi_resolution_last_stats", "satmi_resolution_last_clock", "satmi_dpll_set_split", "satmi_dpll_split_stats",
    "satmi_dp_last_stats",
    "satmi_cdcl_batch_host", "satmi_dpll_set_split_warmup", "satmi_resolution_debug_cand_bytes",
    "satmi_dp_trim", "satmi_resolution_trim", "satmi_cdcl_last_stats", "satmi_launch_chain_floor",
    "satmi_dpll_split_busy",
)


def trim_workspaces():
    """Free the idle Davis-Putnam / resolution device workspaces kept between calls."""
    check(load().satmi_dp_trim(), "satmi_dp_trim")
    check(load().satmi_resolution_trim(), "satmi_resolution_trim")


def set_kernel(policy):
    """Process-wide DPLL kernel policy (KERNEL_AUTO / KERNEL_GENERAL / KERNEL_SCAN / KERNEL_INC)."""
    check(load().satmi_dpll_set_kernel(int(policy)), "satmi_dpll_set_kernel")


SPLIT_OFF, SPLIT_AUTO, SPLIT_ALWAYS = 0, 1, 2


def set_split(enable, helpers_per_cu=0):
    """Process-wide branch splitting of the clause kernels' launch tails: False/SPLIT_OFF,
    True/SPLIT_AUTO (default: launches with at least 1 and at most 8 instances per resident wave) or
    SPLIT_ALWAYS; helpers_per_cu 0 = the library default."""
    check(load().satmi_dpll_set_split(int(enable), int(helpers_per_cu)), "satmi_dpll_set_split")


def set_split_warmup(nodes=-1):
    """Nodes a search visits before it may donate a branch (-1 = the library default)."""
    check(load().satmi_dpll_set_split_warmup(int(nodes)), "satmi_dpll_set_split_warmup")


def split_stats(stream=None):
    """Branch-splitting statistics of the last split launch on `stream` (a HIP stream handle)."""
    out = (ctypes.c_int64 * 7)()
    check(load().satmi_dpll_split_stats(stream, out), "satmi_dpll_split_stats")
    keys = ("donations", "tickets", "claims", "reclaims", "helpers", "handoffs", "done")
    return dict(zip(keys, list(out)))


def split_busy(stream=None):
    """Wave ticks the waves of the last split DPLL launch on `stream` spent searching (0: it did not split)."""
    out = ctypes.c_int64(0)
    check(load().satmi_dpll_split_busy(stream, ctypes.byref(out)), "satmi_dpll_split_busy")
    return out.value


class SatmiError(RuntimeError):
    pass


_lib = None


def load():
    """Load libsatmi.so (once).  torch is imported first when available so that
    the process has exactly one HIP runtime (torch's libamdhip64.so.7 satisfies
    the library's NEEDED entry)."""
    global _lib
    if _lib is not None:
        return _lib
    try:
        import torch  # noqa: F401  (shares its HIP runtime with libsatmi)
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise SatmiError(f"{LIB_PATH} is missing: build it with `make -C {os.path.dirname(_HERE)}` "
                         "(or __graft_entry__.build()); there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    i32p, i64p, vp = P(ctypes.c_int32), P(ctypes.c_int64), ctypes.c_void_p
    L.satmi_abi_version.restype = ctypes.c_int
    L.satmi_last_error.restype = ctypes.c_char_p
    L.satmi_device_count.argtypes = [P(ctypes.c_int)]
    L.satmi_set_device.argtypes = [ctypes.c_int]
    L.satmi_malloc.argtypes = [P(ctypes.c_void_p), ctypes.c_uint64]
    L.satmi_free.argtypes = [vp]
    L.satmi_memcpy_h2d.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.satmi_memcpy_d2h.argtypes = [vp, vp, ctypes.c_uint64, vp]
    L.satmi_stream_synchronize.argtypes = [vp]
    L.satmi_dpll_lds_bytes.restype = ctypes.c_uint64
    L.satmi_dpll_lds_bytes.argtypes = [ctypes.c_int] * 3
    L.satmi_dpll_scan_lds_bytes.restype = ctypes.c_uint64
    L.satmi_dpll_scan_lds_bytes.argtypes = [ctypes.c_int] * 4
    L.satmi_dpll_set_kernel.argtypes = [ctypes.c_int]
    L.satmi_dpll_set_split.argtypes = [ctypes.c_int, ctypes.c_int]
    L.satmi_dpll_split_stats.argtypes = [vp, i64p]
    L.satmi_dpll_split_busy.argtypes = [vp, i64p]
    L.satmi_dpll_set_split_warmup.argtypes = [ctypes.c_int]
    L.satmi_dpll_launch_span.argtypes = [vp, vp]
    L.satmi_wallclock_hz.argtypes = [P(ctypes.c_double)]
    L.satmi_dpll_plan.argtypes = [ctypes.c_int] * 6 + [P(ctypes.c_int), P(ctypes.c_uint64), P(ctypes.c_int)]
    L.satmi_dpll_batch_device.argtypes = [
        ctypes.c_int, vp, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
        ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_int, ctypes.c_int,
        vp, vp, vp, vp, vp, vp, vp]
    L.satmi_dpll_batch_host.argtypes = [
        ctypes.c_int, i32p, i32p, i32p, i32p, i32p, i32p,
        ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_int, ctypes.c_int,
        i32p, i64p, i32p, i32p, i32p, i32p]
    L.satmi_resolution_host.argtypes = [
        ctypes.c_int, i32p, i32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
        i32p, i32p, i64p, ctypes.c_int, i32p, ctypes.c_int64, i64p, ctypes.c_int64, i64p, ctypes.c_int]
    L.satmi_resolution_debug_slot_base.argtypes = [ctypes.c_int64]
    L.satmi_resolution_debug_cand_bytes.argtypes = [ctypes.c_int64]
    L.satmi_cdcl_last_stats.argtypes = [P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_int)]
    L.satmi_dp_last_stats.argtypes = [i64p, i64p, i64p, i64p, P(ctypes.c_int), P(ctypes.c_double)]
    L.satmi_cdcl_batch_host.argtypes = [ctypes.c_int, i32p, i32p, i32p, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_double, i32p, i32p, i32p, ctypes.c_int, i64p,
                                        P(ctypes.c_double)]
    L.satmi_resolution_last_stats.argtypes = [i64p, i64p, ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double)]
    L.satmi_resolution_last_clock.argtypes = [ctypes.POINTER(ctypes.c_double)]
    L.satmi_launch_chain_floor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.satmi_dp_host.argtypes = [
        ctypes.c_int, i32p, i32p, ctypes.c_int64, ctypes.c_int64, ctypes.c_double, i32p, i32p, ctypes.c_int, i32p,
        i32p, ctypes.c_int64, i64p, ctypes.c_int64, i64p, ctypes.c_int]
    for name in EXPORTED:
        getattr(L, name)  # AttributeError here = library/header mismatch
    _lib = L
    return L


def wallclock_hz():
    """Rate of the device wall clock (s_memrealtime) that satmi_dpll_launch_span reports in."""
    hz = ctypes.c_double(0.0)
    check(load().satmi_wallclock_hz(ctypes.byref(hz)), "satmi_wallclock_hz")
    return hz.value


def plan(max_vars, max_clauses, max_lits, max_clause_len, mode=MODE_SOUND, has_init=False):
    """(kernel, lds_bytes_per_wave, waves_per_cu) of the launch satmi_dpll_batch_device would make."""
    k, lds, w = ctypes.c_int(0), ctypes.c_uint64(0), ctypes.c_int(0)
    check(load().satmi_dpll_plan(int(max_vars), int(max_clauses), int(max_lits), int(max_clause_len), int(mode),
                                 int(bool(has_init)), ctypes.byref(k), ctypes.byref(lds), ctypes.byref(w)),
          "satmi_dpll_plan")
    return k.value, lds.value, w.value


def check(rc, what):
    if rc != OK:
        msg = load().satmi_last_error()
        raise SatmiError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def require_gpu():
    L = load()
    n = ctypes.c_int(0)
    rc = L.satmi_device_count(ctypes.byref(n))
    if rc != OK or n.value < 1:
        raise SatmiError("no HIP device visible: the satmi solvers run on MI355X only (no CPU fallback)")
    return n.value


def launch_chain_floor(launches, reps=20):
    """Microseconds per launch of a chain of `launches` dependent one-block
    kernels replayed from a HIP graph (satmi_launch_chain_floor)."""
    L = load()
    require_gpu()
    us = ctypes.c_double(0.0)
    check(L.satmi_launch_chain_floor(int(launches), int(reps), ctypes.byref(us)), "satmi_launch_chain_floor")
    return us.value
