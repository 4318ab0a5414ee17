"""CPU: the drop-in boundary -- the C-ABI library and the C++ shim load and
export exactly what include/*.h declares; without a GPU they fail loudly."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from pip_amd import _lib

ROOT = Path(__file__).resolve().parents[1]

PIP_MANGLED = [  # SURVEY.md 8b, measured from the reference object
    "_Z21pip_standard_checksumPKvjj",
    "_Z15pip_ip_checksumPKvj",
    "_Z17pip_inet_checksumPKvh7in_addrS1_t",
    "_Z18pip_inet6_checksumPKvh8in6_addrS1_t",
    "_Z21pip_inet_checksum_bufSt10shared_ptrI7pip_bufEh7in_addrS2_",
    "_Z22pip_inet6_checksum_bufSt10shared_ptrI7pip_bufEh8in6_addrS2_",
    "_Z15pip_fold_uint32j",
]


def header_functions(path: Path) -> list[str]:
    text = re.sub(r"/\*.*?\*/", "", path.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w \*]*?\b(pipck_\w+)\s*\(", text, flags=re.M)))


def dynsyms(path: Path) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_libpipck_exports_every_declared_function():
    declared = header_functions(ROOT / "include" / "pipck.h")
    assert len(declared) >= 20
    syms = dynsyms(_lib.LIBPIPCK)
    missing = [f for f in declared if f not in syms]
    assert not missing, missing
    # and the ctypes table covers the header exactly
    assert sorted(_lib.SIGNATURES) == declared


def test_internal_tuning_hook_is_outside_the_public_header():
    internal = header_functions(ROOT / "pip_amd" / "csrc" / "pipck_testing.h")
    assert internal == sorted(_lib.INTERNAL_SIGNATURES) == ["pipck_last_launch", "pipck_trace_tasks", "pipck_tune",
                                                            "pipck_tune_probes", "pipck_tune_ring",
                                                            "pipck_tune_xcd_weights"]
    for f in internal:
        assert f in dynsyms(_lib.LIBPIPCK)  # still exported, for tests/ and tools/


def test_public_header_has_no_process_global_knobs():
    """Every mode switch in include/*.h is per context or per queue: a
    declaration whose name speaks of tuning or zero-copy must take a
    pipck_ctx* / pipck_txq* first; nothing reads a knob from the environment
    except a new context's initial per-packet mode."""
    for h in ("pipck.h", "pip_checksum_amd.h"):
        text = re.sub(r"/\*.*?\*/|//[^\n]*", "", (ROOT / "include" / h).read_text(), flags=re.S)
        for name, params in re.findall(r"\b(pip\w*(?:tune|zero_copy|capture)\w*)\s*\(([^)]*)\)", text):
            if h == "pipck.h":
                assert re.match(r"\s*(const\s+)?pipck_(ctx|txq)\s*\*", params), (name, params)
            else:  # the drop-in's switches are per calling thread (thread_local queue)
                assert name.startswith("pip_checksum_amd_"), name
        assert "pipck_tune" not in text and "pipck_host_zero_copy" not in text


def test_product_sources_read_no_environment():
    """No product source reads a knob from the environment: every mode is a
    per-context / per-queue call.  The internal tuning
    hook (pipck_testing.h) is the only process-global switch, and it is not
    read from the environment either."""
    csrc = ROOT / "pip_amd" / "csrc"
    files = sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.cpp")) + sorted(csrc.glob("*.hpp")) + \
        sorted((ROOT / "include").glob("*.h"))
    assert len(files) >= 9
    for f in files:
        code = re.sub(r"/\*.*?\*/|//[^\n]*", "", f.read_text(), flags=re.S)
        assert not re.search(r"\b(getenv|secure_getenv|environ)\b", code), f.name
    # and the documented knobs that used to be environment variables are gone from the headers
    for h in ("pipck.h", "pip_checksum_amd.h"):
        text = (ROOT / "include" / h).read_text()
        for knob in ("PIPCK_HOST_ZERO_COPY", "PIPCK_RESIDENT_VRAM", "PIPCK_TXQ_INPLACE_MAX"):
            assert knob not in text, (h, knob)


def test_libpipck_loads_and_reports_version():
    lib = _lib.load()
    text = (ROOT / "include" / "pipck.h").read_text()
    major = int(re.search(r"#define PIPCK_VERSION_MAJOR (\d+)", text).group(1))
    minor = int(re.search(r"#define PIPCK_VERSION_MINOR (\d+)", text).group(1))
    assert lib.pipck_version() == (major << 16 | minor) and major == 1 and minor >= 2
    assert lib.pipck_cfg_seed(5) == 0x9E3779B97F4A7C15 ^ 5


def test_kernels_are_built_for_gfx950_only():
    blob = _lib.LIBPIPCK.read_bytes()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"gfx1100"):
        assert b"amdgcn-amd-amdhsa--" + other not in blob


def test_shim_exports_pip_mangled_names():
    syms = dynsyms(_lib.LIBSHIM)
    assert set(PIP_MANGLED) <= syms
    # the RX batch verifier is extern "C" (include/pip_checksum_amd.h)
    assert "pip_checksum_amd_verify_packets" in syms and "pip_checksum_amd_rx_abi" in syms
    # the RX verdict meaning (7 = verified) is versioned, in the header and in the library
    shim = C.CDLL(str(_lib.LIBSHIM))
    shim.pip_checksum_amd_rx_abi.restype = C.c_uint32
    assert shim.pip_checksum_amd_rx_abi() == 2
    assert "#define PIP_CHECKSUM_AMD_RX_ABI 2" in (ROOT / "include" / "pip_checksum_amd.h").read_text()
    needed = subprocess.run(["readelf", "-d", str(_lib.LIBSHIM)], check=True, capture_output=True, text=True).stdout
    assert "libpipck.so" in needed


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    lib = _lib.load()
    ctx = C.c_void_p()
    rc = lib.pipck_ctx_create(-1, C.byref(ctx))
    assert rc == _lib.PIPCK_ENODEV
    assert b"no HIP device" in lib.pipck_last_error()
    from pip_amd import engine

    with pytest.raises(RuntimeError):
        engine.require_gpu()
    # the per-packet API has no host path either
    from pip_amd import checksum

    with pytest.raises(_lib.PipckError):
        checksum.pip_ip_checksum(bytes(20))


def test_shim_aborts_without_gpu():
    """pip's API has no error channel: the drop-in prints and aborts rather than
    computing anywhere else (pip_checksum_shim.cpp)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    prog = ROOT / "oracle" / "_ref" / "stack_replay_amd"
    if not prog.exists():
        pytest.skip("replay driver not built (needs /root/reference)")
    r = subprocess.run([str(prog)], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert "libpip_checksum_amd" in r.stderr


def test_batch_abi_rejects_out_of_domain_arguments():
    lib = _lib.load()
    # len > 65535 is outside the batch domain -> ERANGE before anything launches
    rc = lib.pipck_checksum_fixed(C.c_void_p(16), 70000, 70000, 1, None, 1, None, 0, C.c_void_p(16), None)
    assert rc == _lib.PIPCK_ERANGE
    rc = lib.pipck_checksum_fixed(None, 16, 16, 1, None, 1, None, 0, C.c_void_p(16), None)
    assert rc == _lib.PIPCK_EINVAL
    assert lib.pipck_checksum_fixed(None, 16, 16, 0, None, 1, None, 0, None, None) == _lib.PIPCK_OK


@pytest.mark.parametrize("args,why", [
    # (stride, cover_off, cover_len, ck_off, edit_off, edit_len, pseudo_old, pseudo_new)
    ((24, 0, 20, 11, 12, 4, None, None), "odd checksum offset"),
    ((24, 0, 20, 10, 13, 4, None, None), "odd edit offset"),
    ((24, 0, 20, 10, 12, 3, None, None), "odd edit inside the cover"),
    ((24, 0, 20, 10, 8, 4, None, None), "edit overlaps the field"),
    ((24, 0, 20, 10, 18, 4, None, None), "edit past the cover"),
    ((24, 6, 20, 10, 12, 4, None, None), "cover past the stride"),
    ((24, 0, 20, 10, 12, 4, C.c_void_p(16), None), "one pseudo table"),
    ((70000, 0, 65536, 10, 12, 4, None, None), "cover_len out of domain"),
])
def test_update_rejects_bad_geometry(args, why):
    lib = _lib.load()
    stride, cover_off, cover_len, ck_off, edit_off, edit_len, po, pn = args
    rc = lib.pipck_update_fixed(C.c_void_p(16), stride, 1, cover_off, cover_len, ck_off, edit_off, edit_len,
                                C.c_void_p(16), 8, po, pn, 1, None, 0, None)
    assert rc == _lib.PIPCK_EINVAL, why
    assert b"pipck_update_fixed" in lib.pipck_last_error()
