"""ctypes binding of libdfmi.so (the C ABI in include/dfmi.h).

The library is built in-tree (deepfmkit_amd/libdfmi.so, see __graft_entry__.build
or `make -C deepfmkit_amd`). There is NO CPU fallback: if the library or a GPU
is missing, every compute call raises DFMIError.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import sys
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libdfmi.so")

DFMI_MEM_HOST = 0
DFMI_MEM_DEVICE = 1
MAX_LAMBDA = 16

SYMBOLS = ("dfmi_lm_config_default", "dfmi_demod", "dfmi_lm", "dfmi_nls_record", "dfmi_ekf",
           "dfmi_detect_period", "dfmi_device_count", "dfmi_last_error", "dfmi_version", "dfmi_set_tuning",
           "dfmi_last_demod_kernel", "dfmi_qi_row_stride", "dfmi_qi_row_dc", "dfmi_demod_rows",
           "dfmi_probe_read", "dfmi_get_tuning", "dfmi_txt_parse_header", "dfmi_txt_shape", "dfmi_txt_read",
           "dfmi_fit_txt_write", "dfmi_py_repr", "dfmi_txt_last_error", "dfmi_wdfmi_fit", "dfmi_ekf_fit",
           "dfmi_record_moments", "dfmi_synth_asd", "dfmi_synth_snr", "dfmi_bessel_eval",
           "dfmi_release_workspaces", "dfmi_step_timing", "dfmi_step_timing_read", "dfmi_ekf_pit_passes",
           "dfmi_ekf_pit_trace")


class DFMIError(RuntimeError):
    pass


class LMConfig(ctypes.Structure):
    """Mirror of dfmi_lm_config (include/dfmi.h)."""
    _fields_ = [
        ("max_lma_steps", ctypes.c_int32),
        ("n_lambda", ctypes.c_int32),
        ("lambdas", ctypes.c_double * MAX_LAMBDA),
        ("min_step_norm", ctypes.c_double),
        ("conv_improve", ctypes.c_double),
        ("conv_param_change", ctypes.c_double),
        ("fitok_threshold", ctypes.c_double),
        ("m_grid_min", ctypes.c_double),
        ("m_grid_max", ctypes.c_double),
        ("m_grid_step", ctypes.c_double),
        ("bessel_amp_threshold", ctypes.c_double),
        ("sincos_amp_threshold", ctypes.c_double),
    ]


class WdfmiConfig(ctypes.Structure):
    """Mirror of dfmi_wdfmi_config (include/dfmi.h)."""
    _fields_ = [
        ("method", ctypes.c_int32),
        ("ndata", ctypes.c_int32),
        ("ndata_psi", ctypes.c_int32),
        ("period", ctypes.c_int32),
        ("f_samp", ctypes.c_double),
        ("f_mod", ctypes.c_double),
        ("df", ctypes.c_double),
        ("f_ref", ctypes.c_double),
        ("tau_init", ctypes.c_double),
        ("init_a", ctypes.c_double),
        ("init_phi", ctypes.c_double),
        ("init_psi", ctypes.c_double),
    ]


class SnrParams(ctypes.Structure):
    """Mirror of dfmi_snr_params (include/dfmi.h)."""
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("stream", ctypes.c_uint32),
        ("period", ctypes.c_int32),
        ("f_samp", ctypes.c_double),
        ("f_mod", ctypes.c_double),
        ("amp", ctypes.c_double),
        ("visibility", ctypes.c_double),
        ("m", ctypes.c_double),
        ("phi", ctypes.c_double),
        ("psi", ctypes.c_double),
        ("noise_std", ctypes.c_double),
    ]


WDFMI_METHODS = {"wdfmi_nls": 0, "wdfmi_ortho": 1, "wdfmi_seq": 2, "hwdfmi": 3}

_lock = threading.Lock()
_lib = None
RUNTIME = None  # the HIP runtime file libdfmi.so was bound to (set by load())


def _torch_hip_runtime():
    """Path of the HIP runtime PyTorch ships (torch/lib/libamdhip64.so), found WITHOUT
    importing torch; None when torch is absent or is not a ROCm build."""
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.origin:
        return None
    p = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    return p if os.path.exists(p) else None


def _elf_dynamic_strings(path, tag):
    """The DT_SONAME (tag 14) or DT_NEEDED (tag 1) strings of a 64-bit little-endian ELF
    shared object, read from its section headers (no tool, no import); [] if unreadable."""
    import struct
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return []
    if data[:4] != b"\x7fELF" or data[4] != 2 or data[5] != 1:
        return []
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    out = []
    for sec in secs:
        if sec[1] != 6:  # SHT_DYNAMIC
            continue
        strtab = secs[sec[6]]  # sh_link: its string table
        for off in range(sec[4], sec[4] + sec[5], 16):
            d_tag, d_val = struct.unpack_from("<qQ", data, off)
            if d_tag == 0:
                break
            if d_tag == tag:
                s = strtab[4] + d_val
                out.append(data[s:data.index(b"\0", s)].decode())
    return out


def _bind_runtime():
    """Pick the HIP runtime libdfmi.so binds to, before loading it.

    libdfmi.so needs libamdhip64.so.7 (RUNPATH /opt/rocm/lib). PyTorch-ROCm ships its own copy
    (torch/lib/libamdhip64.so, same soname) and its libraries ask for it by the unversioned
    name, so if libdfmi.so is loaded first and torch imported later, the process maps TWO HIP
    and two HSA runtimes (/proc/self/maps), both driving /dev/kfd: whichever initialises first
    holds the device and the other reports no GPU (r04za: torch.cuda.is_available() False
    after a host-memory EKF call). One runtime per process is the fix:
      - torch already imported: its runtime is mapped and the soname match binds to it;
      - torch installed but not imported: torch's runtime FILE is loaded by path (torch itself
        is not imported: no import cost, no import failure), libdfmi.so binds to it by soname,
        and a later `import torch` finds the same file already mapped (glibc matches it by
        device and inode) instead of mapping a second runtime;
      - no torch, or DFMI_HIP_RUNTIME=system: the system runtime /opt/rocm/lib (what the
        numpy + ctypes binding of INTEGRATION.md §B gets).
    Returns the path of the runtime file that will be used, or None for the system one."""
    global RUNTIME
    if os.environ.get("DFMI_HIP_RUNTIME", "") == "system":
        return None
    if "torch" in sys.modules:
        RUNTIME = _torch_hip_runtime()
        return RUNTIME
    p = _torch_hip_runtime()
    if p is None:
        return None
    # preload torch's runtime only when it is the one libdfmi.so asks for: its soname must be
    # libdfmi.so's DT_NEEDED HIP runtime (a torch built against another ROCm major ships another
    # soname; preloading it would map a second runtime, the failure this avoids)
    need = [n for n in _elf_dynamic_strings(LIB_PATH, 1) if n.startswith("libamdhip64")]
    have = _elf_dynamic_strings(p, 14)
    if not need or not have or have[0] not in need:
        import warnings
        warnings.warn(f"deepfmkit_amd: torch's HIP runtime {p} (soname {have}) is not the one libdfmi.so needs "
                      f"({need}); using the system runtime — import torch only if it binds the same one")
        return None
    try:
        ctypes.CDLL(p)
    except OSError:
        return None
    RUNTIME = p
    return p


def load():
    """Load libdfmi.so once (lazy: HIP itself is initialised on the first compute call)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise DFMIError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        _bind_runtime()
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i64, i32, dbl = ctypes.c_int64, ctypes.c_int32, ctypes.c_double
        lib.dfmi_lm_config_default.argtypes = [ctypes.POINTER(LMConfig)]
        lib.dfmi_lm_config_default.restype = None
        lib.dfmi_demod.argtypes = [P, i64, i64, i32, i32, dbl, i32, P, P, i32, P]
        lib.dfmi_demod.restype = ctypes.c_int
        lib.dfmi_lm.argtypes = [P, i64, i32, P, i32, i64, ctypes.POINTER(LMConfig), P, P, P, i32, P]
        lib.dfmi_lm.restype = ctypes.c_int
        lib.dfmi_nls_record.argtypes = [P, i64, i64, i64, i32, i32, dbl, i32, P, i32, i64,
                                        ctypes.POINTER(LMConfig), P, P, i32, P]
        lib.dfmi_nls_record.restype = ctypes.c_int
        lib.dfmi_ekf.argtypes = [P, i64, i64, i64, P, P, P, P, dbl, dbl, i32, i64, P, i32, P]
        lib.dfmi_ekf.restype = ctypes.c_int
        lib.dfmi_ekf_fit.argtypes = [P, i64, i64, i64, P, P, P, P, dbl, dbl, i32, i64, P, i32, P]
        lib.dfmi_ekf_fit.restype = ctypes.c_int
        lib.dfmi_ekf_pit_passes.argtypes = [P, i64]
        lib.dfmi_ekf_pit_passes.restype = ctypes.c_int
        lib.dfmi_ekf_pit_trace.argtypes = [P, i64, i32]
        lib.dfmi_ekf_pit_trace.restype = ctypes.c_int
        lib.dfmi_record_moments.argtypes = [P, i64, i64, i64, P, P, i32, P]
        lib.dfmi_record_moments.restype = ctypes.c_int
        lib.dfmi_synth_asd.argtypes = [P, i64, i64, dbl, P, i32, P]
        lib.dfmi_synth_asd.restype = ctypes.c_int
        lib.dfmi_synth_snr.argtypes = [ctypes.POINTER(SnrParams), i64, i64, P, i32, P]
        lib.dfmi_synth_snr.restype = ctypes.c_int
        lib.dfmi_bessel_eval.argtypes = [P, i64, i32, i32, P, i32, P]
        lib.dfmi_bessel_eval.restype = ctypes.c_int
        lib.dfmi_wdfmi_fit.argtypes = [P, i64, i64, i64, i32, P, i64, ctypes.POINTER(WdfmiConfig), P, P, i32, P]
        lib.dfmi_wdfmi_fit.restype = ctypes.c_int
        lib.dfmi_detect_period.argtypes = [dbl, i32, i32]
        lib.dfmi_detect_period.restype = i32
        lib.dfmi_device_count.argtypes = []
        lib.dfmi_device_count.restype = ctypes.c_int
        lib.dfmi_last_error.argtypes = []
        lib.dfmi_last_error.restype = ctypes.c_char_p
        lib.dfmi_set_tuning.argtypes = [ctypes.c_char_p, i64]
        lib.dfmi_set_tuning.restype = ctypes.c_int
        lib.dfmi_version.argtypes = []
        lib.dfmi_version.restype = ctypes.c_char_p
        lib.dfmi_qi_row_stride.argtypes = [i32]
        lib.dfmi_qi_row_stride.restype = ctypes.c_int32
        lib.dfmi_qi_row_dc.argtypes = [i32]
        lib.dfmi_qi_row_dc.restype = ctypes.c_int32
        lib.dfmi_demod_rows.argtypes = [P, i64, i64, i32, i32, dbl, i32, P, i32, P]
        lib.dfmi_demod_rows.restype = ctypes.c_int
        cp = ctypes.c_char_p
        lib.dfmi_txt_parse_header.argtypes = [cp, i32, P]
        lib.dfmi_txt_parse_header.restype = ctypes.c_int
        lib.dfmi_txt_shape.argtypes = [cp, i32, i32, P, P]
        lib.dfmi_txt_shape.restype = ctypes.c_int
        lib.dfmi_txt_read.argtypes = [cp, i32, i32, i32, P, P, i64, i32]
        lib.dfmi_txt_read.restype = ctypes.c_int
        lib.dfmi_fit_txt_write.argtypes = [cp, cp, P, P, P, P, P, P, i64]
        lib.dfmi_fit_txt_write.restype = ctypes.c_int
        lib.dfmi_py_repr.argtypes = [dbl, ctypes.c_char_p, i32]
        lib.dfmi_py_repr.restype = ctypes.c_int
        lib.dfmi_txt_last_error.argtypes = []
        lib.dfmi_txt_last_error.restype = ctypes.c_char_p
        lib.dfmi_get_tuning.argtypes = [ctypes.c_char_p, P]
        lib.dfmi_get_tuning.restype = ctypes.c_int
        lib.dfmi_release_workspaces.argtypes = []
        lib.dfmi_release_workspaces.restype = ctypes.c_int
        lib.dfmi_step_timing.argtypes = [ctypes.c_int32]
        lib.dfmi_step_timing.restype = ctypes.c_int
        lib.dfmi_step_timing_read.argtypes = [P, P, P]
        lib.dfmi_step_timing_read.restype = ctypes.c_int
        lib.dfmi_probe_read.argtypes = [P, i32]
        lib.dfmi_probe_read.restype = ctypes.c_int
        lib.dfmi_last_demod_kernel.argtypes = []
        lib.dfmi_last_demod_kernel.restype = ctypes.c_char_p
        _lib = lib
        return lib


def check(rc, what):
    if rc != 0:
        msg = load().dfmi_last_error().decode(errors="replace")
        raise DFMIError(f"{what} failed ({rc}): {msg}")


def ptr(a):
    """Raw pointer of a numpy array or a torch tensor (data_ptr)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()
