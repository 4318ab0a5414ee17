"""Device-resident batch engine: thin Python over the C ABI of libpipck.so.

PyTorch is plumbing here -- it owns device memory, the current HIP stream and
the multi-process runtime; every byte of checksum work is done by the HIP
kernels in ``pip_amd/csrc``.  Results are host-order u16 (what pip's
functions return before the caller's ``htons``), stored in int16 tensors.

Reference interface mirrored: ``pip/pip_checksum.h:17-34`` -- the batch calls
compute, for every packet of a batch, exactly what ``pip_ip_checksum``,
``pip_inet_checksum``/``pip_inet6_checksum`` or their ``_buf`` chain variants
return for that packet.
"""
from __future__ import annotations

import ctypes as C

from . import _lib
from ._lib import Desc, Flow4, Flow6, call, check, load  # noqa: F401  (re-exported)

DESC_BYTES = C.sizeof(Desc)  # 16: u64 offset, u32 len, u32 flow


def _torch():
    import torch

    return torch


def _ptr(t) -> C.c_void_p | None:
    return None if t is None else C.c_void_p(t.data_ptr())


def current_stream(device=None) -> C.c_void_p:
    torch = _torch()
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_gpu() -> None:
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("pip_amd engine needs a HIP device (gfx950); none is visible")
    load()


_hip = None


def hip_runtime() -> C.CDLL:
    """A handle on THE HIP runtime mapped into this process -- the one libpipck.so
    links and launches through, and whose streams torch hands us.  Opening
    "libamdhip64.so" by its bare name could load a second runtime instance (another
    soname or path); events or queries made through it would not see this
    runtime's streams.  So the library is found in /proc/self/maps after
    libpipck.so is loaded and opened with RTLD_NOLOAD (never a fresh load); more
    than one mapped runtime is an error."""
    global _hip
    if _hip is None:
        import os

        load()
        paths = set()
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 6 and os.path.basename(parts[5]).startswith("libamdhip64.so"):
                    paths.add(os.path.realpath(parts[5]))
        if len(paths) != 1:
            raise RuntimeError(f"expected exactly one HIP runtime mapped in this process, found {sorted(paths)}")
        _hip = C.CDLL(paths.pop(), mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    return _hip


def pci_bus_id(device: int) -> str:
    """PCI bus id of a HIP device ("0000:05:00.0"), from hipDeviceGetPCIBusId: names the physical
    GPU a rank ran on (bench.py's per_rank_device)."""
    buf = C.create_string_buffer(64)
    try:
        if hip_runtime().hipDeviceGetPCIBusId(buf, C.c_int(len(buf)), C.c_int(device)) == 0:
            return buf.value.decode()
    except (OSError, RuntimeError):
        pass
    p = _torch().cuda.get_device_properties(device)
    return f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:" \
           f"{getattr(p, 'pci_device_id', 0):02x}.0"


# ---------------------------------------------------------------- flows
def gen_flows(family: int, n_flows: int, seed: int, proto: int, device=None):
    """Synthetic flow table on the device + its pseudo-header bases."""
    torch = _torch()
    size = C.sizeof(Flow4 if family == 4 else Flow6)
    flows = torch.empty(n_flows * size, dtype=torch.uint8, device=device or "cuda")
    fn = "pipck_gen_flows4" if family == 4 else "pipck_gen_flows6"
    call(fn, _ptr(flows), n_flows, seed, proto, current_stream(flows.device))
    return flows, prepare_flows(family, flows, n_flows)


def prepare_flows(family: int, flows, n_flows: int):
    """flows: device uint8 tensor of n_flows pipck_flow4/pipck_flow6 records."""
    torch = _torch()
    pseudo = torch.empty(n_flows, dtype=torch.int32, device=flows.device)
    fn = "pipck_flows4_prepare" if family == 4 else "pipck_flows6_prepare"
    call(fn, _ptr(flows), n_flows, _ptr(pseudo), current_stream(flows.device))
    return pseudo


def flows_to_device(family: int, flows_bytes: bytes, device=None):
    torch = _torch()
    t = torch.frombuffer(bytearray(flows_bytes), dtype=torch.uint8).to(device or "cuda")
    return t


# ---------------------------------------------------------------- batches
def _n_flows(n_flows, pseudo, flow_of) -> int:
    """The n_flows a bounded (_n) call gets.  Without flow_of it is the modulus of
    (flow_origin + i) % n_flows (default 1); with flow_of it bounds every entry on
    the device (an entry >= n_flows gives that packet 0 and PIPCK_ERANGE), so its
    default is the whole table, pseudo.numel() -- never 1, which would refuse every
    packet whose flow is >= 1."""
    if n_flows is not None:
        return n_flows
    if flow_of is not None and pseudo is not None:
        return pseudo.numel()
    return 1


def checksum_fixed(arena, stride: int, length: int, n: int, pseudo=None, n_flows: int | None = None, flow_of=None,
                   flow_origin: int = 0, out=None, err=None):
    """Fixed-stride batch (pipck_checksum_fixed_n): packet i at arena[i * stride:], `length` bytes.
    flow_of entries are bounded on the device by n_flows (default: the whole pseudo table); an
    entry past it gives that packet 0 and ORs 1 << PIPCK_ERANGE into err (optional device int32)."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    _check_span(arena, stride, length, n)
    call("pipck_checksum_fixed_n", _ptr(arena), stride, length, n, _ptr(pseudo), _n_flows(n_flows, pseudo, flow_of),
         _ptr(flow_of), flow_origin, _ptr(out), _ptr(err), current_stream(arena.device))
    return out


def _bound(fn: str, *args):
    """A zero-argument call of C entry `fn` with its ctypes arguments built once
    (pointers, sizes and the stream fixed): what a C caller of the batch ABI
    pays per batch, without this module's per-call argument handling."""
    f = getattr(load(), fn)

    def run():
        rc = f(*args)
        if rc:
            check(fn, rc)

    return run


def prepare_checksum_fixed(arena, stride: int, length: int, n: int, pseudo=None, n_flows: int | None = None,
                           flow_of=None, flow_origin: int = 0, out=None, err=None):
    """checksum_fixed with its arguments checked and bound once; returns (run, out):
    each run() checksums the batch into out on the current stream.  The tensors
    must stay alive and in place while run is used."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    _check_span(arena, stride, length, n)
    return _bound("pipck_checksum_fixed_n", _ptr(arena), stride, length, n, _ptr(pseudo),
                  _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(out), _ptr(err),
                  current_stream(arena.device)), out


def verify_fixed(arena, stride: int, length: int, n: int, pseudo=None, n_flows: int | None = None, flow_of=None,
                 flow_origin: int = 0, ok=None, err=None):
    """RX verification of a fixed-stride batch (pipck_verify_fixed_n, bounded as checksum_fixed:
    a refused packet verifies as 0)."""
    torch = _torch()
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check_span(arena, stride, length, n)
    call("pipck_verify_fixed_n", _ptr(arena), stride, length, n, _ptr(pseudo), _n_flows(n_flows, pseudo, flow_of),
         _ptr(flow_of), flow_origin, _ptr(ok), _ptr(err), current_stream(arena.device))
    return ok


def checksum_ragged(arena, desc, pseudo=None, out=None, err=None):
    """desc: device int64 tensor (n, 2) laid out as pipck_desc.  Bounded on the device
    (pipck_checksum_ragged_n): a descriptor past the arena, longer than 65535 B or naming a
    flow past `pseudo` gets 0 and ORs 1 << PIPCK_ERANGE into err (optional device int32)."""
    torch = _torch()
    n = desc.shape[0]
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    call("pipck_checksum_ragged_n", _ptr(arena), _nbytes(arena), _ptr(desc), n, _ptr(pseudo),
         pseudo.numel() if pseudo is not None else 0, _ptr(out), _ptr(err), current_stream(arena.device))
    return out


def verify_ragged(arena, desc, pseudo=None, ok=None, err=None):
    """RX verification of a ragged batch whose packets carry their checksum field
    (pipck_verify_ragged_n, bounded as checksum_ragged)."""
    torch = _torch()
    n = desc.shape[0]
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=arena.device)
    call("pipck_verify_ragged_n", _ptr(arena), _nbytes(arena), _ptr(desc), n, _ptr(pseudo),
         pseudo.numel() if pseudo is not None else 0, _ptr(ok), _ptr(err), current_stream(arena.device))
    return ok


def tune_xcd_weights(m=None, period: int = 0) -> None:
    """k_flat's XCD-weighted static deal (pipck_tune_xcd_weights, internal): XCD x keeps
    m[x] of every `period` blocks dealt to it; None / 0 = off."""
    arr = (C.c_uint32 * 8)(*[int(x) for x in m]) if m is not None else None
    call("pipck_tune_xcd_weights", arr, period)


def _nbytes(t) -> int:
    return t.numel() * t.element_size()


def checksum_packed(arena, lens, tile_chunk, n: int | None = None, pseudo=None, n_flows: int | None = None,
                    flow_of=None, flow_origin: int = 0, out=None, err=None):
    """Packed ragged batch (pipck_checksum_packed_n): lens = device int16/uint16 tensor of
    packet lengths, tile_chunk = packed_index(lens); packet i at 16 * (chunks before i).
    The device bounds every tile by the arena's size (err: optional device int32,
    OR-ed with 1 << PIPCK_ERANGE for a tile past it, whose results are then 0) and
    every flow_of entry by n_flows (default: the whole pseudo table, as _n_flows)."""
    torch = _torch()
    n = lens.numel() if n is None else n
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    _check_packed(arena, lens, tile_chunk, n)
    call("pipck_checksum_packed_n", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_chunk), n, _ptr(pseudo),
         _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(out), _ptr(err),
         current_stream(arena.device))
    return out


def verify_packed(arena, lens, tile_chunk, n: int | None = None, pseudo=None, n_flows: int | None = None,
                  flow_of=None, flow_origin: int = 0, ok=None, err=None):
    torch = _torch()
    n = lens.numel() if n is None else n
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check_packed(arena, lens, tile_chunk, n)
    call("pipck_verify_packed_n", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_chunk), n, _ptr(pseudo),
         _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(ok), _ptr(err),
         current_stream(arena.device))
    return ok


def packed_index(lens, n: int | None = None):
    """tile_chunk for a packed batch: u64 (as int64) per 64 packets + the total."""
    torch = _torch()
    n = lens.numel() if n is None else n
    tc = torch.empty((n + 63) // 64 + 1, dtype=torch.int64, device=lens.device)
    call("pipck_packed_index", _ptr(lens), n, _ptr(tc), current_stream(lens.device))
    return tc


_packed_total: dict = {}  # id(tile_chunk) -> (weakref, tensor version, n, chunks)


def _check_packed(arena, lens, tile_chunk, n, unit: int = 16):
    """Host-side guard (the device bounds every tile as well, pipck_*_packed*_n):
    the batch must lie inside the arena.  The index's total
    (tile_chunk[ceil(n/64)], one device read) is cached on the index tensor
    OBJECT and its in-place version counter, never on addresses: a freed tensor's
    address is reused by the caching allocator, and a pointer-keyed cache would
    then skip the check for a larger batch.  The bound itself is re-checked
    against the arena on every call.  An index refilled through a raw pointer
    (a custom kernel writing into a reused tile_off) does not bump _version, so
    this guard can keep its old total; the device bound (the _n calls) still
    refuses every tile past the arena (PIPCK_ERANGE, results 0)."""
    import weakref

    if n > lens.numel() or tile_chunk.numel() < (n + 63) // 64 + 1:
        raise ValueError("lens / tile_chunk shorter than the batch")
    ent = _packed_total.get(id(tile_chunk))
    if ent is not None and ent[0]() is tile_chunk and ent[1] == tile_chunk._version and ent[2] == n:
        chunks = ent[3]
    else:
        chunks = int(tile_chunk[(n + 63) // 64].item())
        if len(_packed_total) > 64:
            _packed_total.clear()
        _packed_total[id(tile_chunk)] = (weakref.ref(tile_chunk), tile_chunk._version, n, chunks)
    need = unit * chunks if unit == 16 else (chunks + 15) // 16 * 16  # bytes: read to the next 16-B boundary
    if need > arena.numel() * arena.element_size():
        raise ValueError(f"packed batch needs {need} B, arena has {arena.numel() * arena.element_size()}")


def checksum_packed_bytes(arena, lens, tile_off, n: int | None = None, pseudo=None, n_flows: int | None = None,
                          flow_of=None, flow_origin: int = 0, out=None, err=None):
    """Byte-packed ragged batch (pipck_checksum_packed_bytes_n): packets back to back with no padding,
    lens = device int16/uint16 lengths, tile_off = packed_bytes_index(lens); arena 128-byte aligned.
    Tiles are bounded by the arena's size on the device (err as checksum_packed)."""
    torch = _torch()
    n = lens.numel() if n is None else n
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    _check_packed(arena, lens, tile_off, n, unit=1)
    call("pipck_checksum_packed_bytes_n", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_off), n, _ptr(pseudo),
         _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(out), _ptr(err),
         current_stream(arena.device))
    return out


def prepare_checksum_packed_bytes(arena, lens, tile_off, n: int | None = None, pseudo=None,
                                  n_flows: int | None = None, flow_of=None, flow_origin: int = 0, out=None, err=None):
    """checksum_packed_bytes with its arguments checked and bound once (as
    prepare_checksum_fixed); returns (run, out)."""
    torch = _torch()
    n = lens.numel() if n is None else n
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=arena.device)
    _check_packed(arena, lens, tile_off, n, unit=1)
    return _bound("pipck_checksum_packed_bytes_n", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_off), n,
                  _ptr(pseudo), _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(out),
                  _ptr(err), current_stream(arena.device)), out


def verify_packed_bytes(arena, lens, tile_off, n: int | None = None, pseudo=None, n_flows: int | None = None,
                        flow_of=None, flow_origin: int = 0, ok=None, err=None):
    torch = _torch()
    n = lens.numel() if n is None else n
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check_packed(arena, lens, tile_off, n, unit=1)
    call("pipck_verify_packed_bytes_n", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_off), n, _ptr(pseudo),
         _n_flows(n_flows, pseudo, flow_of), _ptr(flow_of), flow_origin, _ptr(ok), _ptr(err),
         current_stream(arena.device))
    return ok


def rx_verify_ring(ring, stride: int, lens, n: int | None = None, ok=None, err=None):
    """Received frames in the fixed-size slots of a device ring (pipck_rx_verify_ring_n): the
    PIPCK_RX_* bits per slot (uint8).  A slot length past the stride is refused on the device
    (verdict 0, 1 << PIPCK_ERANGE OR-ed into err, an optional device int32)."""
    torch = _torch()
    n = lens.numel() if n is None else n
    if n * stride > _nbytes(ring) or n > lens.numel():
        raise ValueError("ring smaller than n * stride, or fewer lengths than slots")
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=ring.device)
    call("pipck_rx_verify_ring_n", _ptr(ring), stride, _ptr(lens), n, _ptr(ok), _ptr(err),
         current_stream(ring.device))
    return ok


def rx_verify_device(arena, lens, tile_off, n: int | None = None, ok=None, err=None):
    """Received IP packets in device memory, byte-packed (pipck_rx_verify_device): the
    PIPCK_RX_* bits per packet (uint8), as pipck_rx_verify gives for the same bytes in
    host memory.  Tiles are bounded by the arena's size on the device (err as checksum_packed)."""
    torch = _torch()
    n = lens.numel() if n is None else n
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=arena.device)
    _check_packed(arena, lens, tile_off, n, unit=1)
    call("pipck_rx_verify_device", _ptr(arena), _nbytes(arena), _ptr(lens), _ptr(tile_off), n, _ptr(ok), _ptr(err),
         current_stream(arena.device))
    return ok


def packed_bytes_index(lens, n: int | None = None):
    """tile_off for a byte-packed batch: the byte offset of every 64th packet (u64 as int64) + the total."""
    torch = _torch()
    n = lens.numel() if n is None else n
    to = torch.empty((n + 63) // 64 + 1, dtype=torch.int64, device=lens.device)
    call("pipck_packed_bytes_index", _ptr(lens), n, _ptr(to), current_stream(lens.device))
    return to


def checksum_chains(arena, segs, seg_begin, pkt_flow=None, pseudo=None, out=None, err=None):
    """segs: (n_segs, 2) int64 descriptors; seg_begin: (n_packets+1,) int64 CSR offsets.
    Bounded on the device (pipck_checksum_chains_n): a packet with a segment past the arena,
    a flow past `pseudo` or a segment range outside segs gets 0 and sets err (as checksum_ragged)."""
    torch = _torch()
    n_pk = seg_begin.shape[0] - 1
    scratch = torch.empty(max(segs.shape[0], 1), dtype=torch.int32, device=arena.device)
    if out is None:
        out = torch.empty(n_pk, dtype=torch.int16, device=arena.device)
    call("pipck_checksum_chains_n", _ptr(arena), _nbytes(arena), _ptr(segs), segs.shape[0], _ptr(seg_begin),
         _ptr(pkt_flow), n_pk, _ptr(pseudo), pseudo.numel() if pseudo is not None else 0, _ptr(scratch), _ptr(out),
         _ptr(err), current_stream(arena.device))
    return out


def update_fixed(arena, stride: int, n: int, cover_off: int, cover_len: int, ck_off: int, edit_off: int,
                 edit_len: int, new_bytes=None, new_stride: int = 0, pseudo_old=None, pseudo_new=None,
                 n_flows: int | None = None, flow_of=None, flow_origin: int = 0, err=None) -> None:
    """Rewrite bytes [edit_off, edit_off+edit_len) of every packet with new_bytes[i*new_stride:] and patch
    the big-endian checksum field at ck_off incrementally (RFC 1624); see pipck_update_fixed_n.  A
    flow_of entry >= n_flows (default: the tables' length) leaves its packet untouched and ORs
    1 << PIPCK_ERANGE into err (optional device int32)."""
    if pseudo_old is not None and pseudo_new is not None and pseudo_old.numel() != pseudo_new.numel():
        raise ValueError("pseudo_old and pseudo_new must have the same number of flows")
    _check_span(arena, stride, cover_off + cover_len, n)
    if edit_len and new_bytes is not None and n and \
            (n - 1) * new_stride + edit_len > new_bytes.numel() * new_bytes.element_size():
        raise ValueError("new_bytes is too small for the batch")
    call("pipck_update_fixed_n", _ptr(arena), stride, n, cover_off, cover_len, ck_off, edit_off, edit_len,
         _ptr(new_bytes), new_stride, _ptr(pseudo_old), _ptr(pseudo_new), _n_flows(n_flows, pseudo_old, flow_of),
         _ptr(flow_of), flow_origin, _ptr(err), current_stream(arena.device))


def _check_span(arena, stride, length, n):
    """Host-side guard: the kernels must never read past the arena."""
    if n and (n - 1) * stride + length > arena.numel() * arena.element_size():
        raise ValueError(f"arena of {arena.numel() * arena.element_size()} B is too small for "
                         f"{n} packets x stride {stride} (len {length})")


def make_desc(offsets, lengths, flows, device=None):
    """Pack host arrays into a (n, 2) int64 device tensor of pipck_desc."""
    import numpy as np

    torch = _torch()
    n = len(offsets)
    raw = np.zeros(n, dtype=[("offset", "<u8"), ("len", "<u4"), ("flow", "<u4")])
    raw["offset"], raw["len"], raw["flow"] = offsets, lengths, flows
    return torch.from_numpy(raw.view(np.int64).reshape(n, 2).copy()).to(device or "cuda")


# ---------------------------------------------------------------- generators
def cfg_seed(cfg: int) -> int:
    return load().pipck_cfg_seed(cfg)


def gen_fixed(arena, stride: int, length: int, n: int, first: int, seed: int, hdr: int) -> None:
    _check_span(arena, stride, length, n)
    if n and (n * stride) > arena.numel() * arena.element_size():
        raise ValueError("arena too small for generated stride slots")
    call("pipck_gen_fixed", _ptr(arena), stride, length, n, first, seed, hdr, current_stream(arena.device))


def gen_ragged(n: int, first: int, seed: int, hdr: int, n_flows: int, device=None, lengths=None):
    """Zipf-length batch (cfg4 shape). Returns (arena, desc, lengths)."""
    torch = _torch()
    dev = device or "cuda"
    if lengths is None:
        lengths = torch.empty(n, dtype=torch.int32, device=dev)
        call("pipck_gen_zipf_lengths", _ptr(lengths), n, first, seed, current_stream(lengths.device))
    desc = torch.empty((n, 2), dtype=torch.int64, device=lengths.device)
    nbytes = C.c_uint64(0)
    call("pipck_gen_ragged_layout", _ptr(lengths), n, first, n_flows, _ptr(desc), C.byref(nbytes),
         current_stream(lengths.device))
    arena = torch.empty(max(int(nbytes.value), 16), dtype=torch.uint8, device=lengths.device)
    call("pipck_gen_ragged_fill", _ptr(arena), _ptr(desc), n, first, seed, hdr, current_stream(arena.device))
    return arena, desc, lengths


def gen_packed(n: int, first: int, seed: int, hdr: int, device=None, lengths=None):
    """Zipf-length batch (cfg4 shape) in the packed layout: (arena, lens u16-in-int16, tile_chunk, lengths i32).
    Bytes and layout equal gen_ragged's; only the descriptors are replaced by lengths + a per-64 index."""
    torch = _torch()
    arena, desc, lengths = gen_ragged(n, first, seed, hdr, 1, device=device, lengths=lengths)
    del desc
    lens16 = lengths.to(torch.int16)
    return arena, lens16, packed_index(lens16, n), lengths


def gen_packed_bytes(n: int, first: int, seed: int, hdr: int, device=None, lengths=None):
    """Zipf-length batch (cfg4 shape) in the byte-packed layout: (arena, lens u16-in-int16, tile_off, lengths i32).
    Packet bytes equal gen_ragged's packet for packet; only the 16-byte padding between packets is gone."""
    torch = _torch()
    dev = device or "cuda"
    if lengths is None:
        lengths = torch.empty(n, dtype=torch.int32, device=dev)
        call("pipck_gen_zipf_lengths", _ptr(lengths), n, first, seed, current_stream(lengths.device))
    lens16 = lengths.to(torch.int16)
    tile_off = packed_bytes_index(lens16, n)
    total = int(tile_off[(n + 63) // 64].item())
    arena = torch.empty(max((total + 15) // 16 * 16, 16), dtype=torch.uint8, device=lengths.device)
    arena[total:].zero_()  # the bytes after the last packet, up to the 16-B boundary the kernel reads to
    call("pipck_gen_packed_bytes", _ptr(arena), _ptr(lens16), _ptr(tile_off), n, first, seed, hdr,
         current_stream(arena.device))
    return arena, lens16, tile_off, lengths


def gen_rx_ring(n: int, seed: int, stride: int, l4_len: int = 0):
    """gen_rx_frames laid out in the fixed-size slots of a receive ring: frame i at
    ring[i * stride], the rest of each slot zero (pipck_rx_verify_ring's layout).
    l4_len > 0: every frame's L4 length (a dense ring), else cfg4's Zipf lengths.
    Returns (ring, lens u16-in-int16, kind)."""
    torch = _torch()
    arena, lens, _, kind, start, l4 = gen_rx_frames(n, seed, l4_len=l4_len)
    ln = lens.to(torch.int64) & 0xFFFF
    if int(ln.max().item()) > stride:
        raise ValueError("a frame is longer than the slot stride")
    ring = torch.zeros(n * stride, dtype=torch.uint8, device=arena.device)
    step = 1 << 16  # frames per copy pass (bounded index tensors)
    for f0 in range(0, n, step):
        lc, sc = ln[f0:f0 + step], start[f0:f0 + step]
        m = lc.numel()
        frame = torch.repeat_interleave(torch.arange(m, device=arena.device), lc)
        excl = torch.cumsum(lc, 0) - lc
        within = torch.arange(frame.numel(), device=arena.device) - excl[frame]
        ring[(f0 + frame) * stride + within] = arena[sc[frame] + within]
    return ring, lens, kind


def gen_rx_frames(n: int, seed: int, checksummed: bool = True, l4_len: int = 0):
    """Received-frame batch for pipck_rx_verify_device (bench and tests; synthetic):
    n frames back to back, cfg4's Zipf L4 lengths (64-9,000 B; l4_len > 0: all that
    length) under an IPv4 (kinds
    0, 1: TCP; 2: UDP) or IPv6 (kind 3: TCP) header, every other byte random.  With
    `checksummed`, the TCP/UDP and IPv4 header checksum fields are filled in by this
    engine's own batch kernels (pipck_checksum_ragged over the L4 segments with each
    frame's pseudo-header, then over the 20-byte IPv4 headers), as a sender would,
    so every frame verifies except UDP/IPv4 ones whose checksum came out 0x0000 (sent
    as "no checksum", RFC 768).  Returns (arena, lens u16-in-int16, tile_off, kind,
    start, l4_len) with start / l4_len int64 on the device."""
    torch = _torch()
    g = torch.Generator(device="cuda").manual_seed(seed)
    l4 = torch.empty(n, dtype=torch.int32, device="cuda")
    if l4_len:
        l4.fill_(l4_len)
    else:
        call("pipck_gen_zipf_lengths", _ptr(l4), n, 0, cfg_seed(4), current_stream())
    kind = torch.randint(0, 4, (n,), device="cuda", generator=g)
    v6 = kind == 3
    hl = torch.where(v6, 40, 20).to(torch.int64)
    l4 = l4.to(torch.int64)
    frame = l4 + hl
    lens = frame.to(torch.int16)
    tile_off = packed_bytes_index(lens)
    total = int(tile_off[-1].item())
    arena = torch.randint(0, 256, ((total + 16 + 127) // 128 * 128,), dtype=torch.uint8, device="cuda", generator=g)
    start = torch.cumsum(frame, 0) - frame
    proto = torch.where(kind == 2, 17, 6)

    def put(col, val, mask):
        idx = (start + col)[mask]
        arena[idx] = (val[mask] if torch.is_tensor(val) else torch.full_like(idx, val)).to(torch.uint8)

    v4 = ~v6
    put(0, 0x45, v4)
    put(2, frame >> 8, v4)
    put(3, frame & 0xFF, v4)
    put(6, 0, v4)  # not a fragment
    put(7, 0, v4)
    put(9, proto, v4)
    put(0, 0x60, v6)
    put(4, l4 >> 8, v6)
    put(5, l4 & 0xFF, v6)
    put(6, 6, v6)
    if not checksummed:
        return arena, lens, tile_off, kind, start, l4
    field = start + hl + torch.where(proto == 6, 16, 6)  # th_sum / uh_sum
    for k in (0, 1):
        arena[field + k] = 0
    put(10, 0, v4)
    put(11, 0, v4)

    def be_words(first, count):  # big-endian 16-bit words of [start + first, + 2 * count) summed
        idx = start[:, None] + first + torch.arange(2 * count, device="cuda")
        b = arena[idx].to(torch.int64)
        return (b[:, 0::2] * 256 + b[:, 1::2]).sum(1)

    pseudo = torch.where(v6, be_words(8, 16), be_words(12, 4)) + proto  # addresses + proto (pip_checksum.cpp:45-82)
    flows = torch.arange(n, device="cuda", dtype=torch.int64)

    def ragged(off, ln, ps):
        desc = torch.stack([off, ln | (flows << 32)], 1)
        return checksum_ragged(arena, desc, ps).to(torch.int64) & 0xFFFF

    r = ragged(start + hl, l4, pseudo.to(torch.int32))
    arena[field] = (r >> 8).to(torch.uint8)
    arena[field + 1] = (r & 0xFF).to(torch.uint8)
    ip = ragged(start, torch.full_like(l4, 20), None)
    put(10, ip >> 8, v4)
    put(11, ip & 0xFF, v4)
    return arena, lens, tile_off, kind, start, l4


def tune(lanes_per_packet: int = 0, loads_per_lane: int = 0, blocks: int = 0, plain_loads: bool = False,
         flat: bool = True, nt_loads: bool = False, rows_per_task: int = 0, xcd_groups: bool = False,
         packed_tiles: bool = True, wide_blocks: bool = False,
         small: bool = True, small_k_log: int = 0, flat_small: bool = True, tiny_tiles: bool = True,
         flat_tiny: bool = True, force_flat_tiny: bool = False, packed_marks_only: bool = False,
         trace: bool = False, loads_only: bool = False, no_task_end: bool = False,
         end_no_store: bool = False, alt_flat_schedule: bool = False,
         plain_result_stores: bool = False, wave_stores: bool = False, free_run: bool = False,
         packed_no_align: bool = False, hdr_in_place: bool = False, ring_own_slots: bool = False,
         ring_all_coop: bool = False, ring_adapt: bool | None = None) -> None:
    """Process-wide launch-shape override (0 = automatic) for tests and tools: the internal pipck_tune
    (pip_amd/csrc/pipck_testing.h), not part of the public ABI.  Every setting computes the same results
    except the measurement-only probes loads_only (bit 21), no_task_end (22), end_no_store (23) and
    hdr_in_place (pipck_tune_probes bit 0, not a tune flag: k_hdr stores the results into the headers'
    ip_sum and leaves the result array untouched).  alt_flat_schedule (bit 28) never changes results.
    ring_own_slots / ring_all_coop: k_ring's row stream never / always deals items round-robin to the
    block's waves; ring_adapt: None = automatic (jumbo slots take k_ring or the row stream by the
    feedback of the ring's earlier launches), False = k_ring at every fill, True = the feedback at every
    stride -- pipck_tune_ring's own word, apart from the flags above (they once shared bits
    27 / 29 with small_k_log and plain_result_stores)."""
    if not 0 <= small_k_log <= 4:
        raise ValueError("small_k_log must be 0..4")
    flags = ((1 if plain_loads else 0) | (0 if flat else 2) | (4 if nt_loads else 0) | (8 if xcd_groups else 0)
             | (0 if packed_tiles else 16) | (32 if wide_blocks else 0) | (0 if small else 64)
             | (0 if flat_small else 128) | (rows_per_task << 8) | (0 if tiny_tiles else 1 << 16)
             | (0 if flat_tiny else 1 << 17) | (1 << 18 if force_flat_tiny else 0) | (small_k_log << 24)
             | (1 << 19 if packed_marks_only else 0) | (1 << 20 if trace else 0) | (1 << 21 if loads_only else 0) | (1 << 22 if no_task_end else 0)
             | (1 << 23 if end_no_store else 0) | (1 << 28 if alt_flat_schedule else 0)
             | (1 << 29 if plain_result_stores else 0)
             | (1 << 30 if (wave_stores or packed_no_align) else 0)
             | (1 << 31 if free_run else 0))
    load().pipck_tune(lanes_per_packet, loads_per_lane, blocks, flags)
    load().pipck_tune_probes(1 if hdr_in_place else 0)
    ring = (1 if ring_own_slots else 0) | (2 if ring_all_coop else 0) | {None: 0, False: 4, True: 8}[ring_adapt]
    if ring or hasattr(load(), "pipck_tune_ring"):  # (a pre-1.3 build under PIPCK_LIB has no ring word)
        load().pipck_tune_ring(ring)
