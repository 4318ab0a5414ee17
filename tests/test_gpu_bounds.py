"""GPU: the packed-batch C ABI bounds every tile by the arena on the device
(pipck_{checksum,verify}_packed{,_bytes}_n, include/pipck.h) -- VERDICT r03 item 5.

The calls go straight through ctypes, with no Python-side guard: an index that
places a tile (64 packets) past the arena -- a stale or foreign tile_off /
tile_chunk, or lengths that no longer match it -- must read nothing there,
report PIPCK_ERANGE in d_err and give 0 for that tile's packets, while every
other tile's results stay those of the untampered batch."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from pip_amd import _lib, engine  # noqa: E402
from pip_amd.workloads import CFG4, N_FLOWS  # noqa: E402

pytestmark = pytest.mark.gpu
ERANGE_BIT = 1 << 2  # 1 << PIPCK_ERANGE


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _run(fn, arena, arena_bytes, lens, index, n, pseudo, verify):
    lib = _lib.load()
    out = torch.zeros(n, dtype=torch.uint8 if verify else torch.int16, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = getattr(lib, fn)(_p(arena), C.c_uint64(arena_bytes), _p(lens), _p(index), C.c_uint64(n), _p(pseudo),
                          C.c_uint32(N_FLOWS), C.c_void_p(0), C.c_uint64(0), _p(out), _p(err), C.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, _lib.load().pipck_last_error()
    return out.cpu().numpy().view(np.uint8 if verify else np.uint16), int(err.item())


@pytest.mark.parametrize("layout", ["bytes", "packed16"])
@pytest.mark.parametrize("verify", [False, True])
def test_index_past_the_arena_is_an_error_not_a_fault(layout, verify):
    n = 64 * 40 + 17  # 41 tiles, the last one partial
    w = CFG4
    if layout == "bytes":
        arena, lens, index, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_bytes_n" if verify else "pipck_checksum_packed_bytes_n"
        unit = 1
    else:
        arena, lens, index, _ = engine.gen_packed(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_n" if verify else "pipck_checksum_packed_n"
        unit = 16
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    nbytes = arena.numel()
    good, err0 = _run(fn, arena, nbytes, lens, index, n, pseudo, verify)
    assert err0 == 0
    if not verify:  # the bounded call equals the plain (trusted-index) one on a correct index
        plain = (engine.checksum_packed_bytes if layout == "bytes" else engine.checksum_packed)(
            arena, lens, index, n, pseudo, N_FLOWS)
        assert np.array_equal(plain.cpu().numpy().view(np.uint16), good)
    total = int(index[(n + 63) // 64].item())  # bytes (or chunks) of the whole batch
    bad = index.clone()
    bad[5] = total * 1000 + 12345            # far past the arena
    bad[9] = total - 3                        # starts inside, its packets run past the end
    bad[13] = (1 << 62) + 7                   # would overflow an unchecked offset + length
    got, err = _run(fn, arena, nbytes, lens, bad, n, pseudo, verify)
    assert err == ERANGE_BIT
    flagged = np.zeros(n, dtype=bool)
    for t in (5, 9, 13):
        flagged[64 * t:64 * t + 64] = True
    assert (got[flagged] == 0).all()
    assert np.array_equal(got[~flagged], good[~flagged])
    # an arena shorter than the index claims: the tail tiles are refused the same way
    short = (total * unit) // 2
    got, err = _run(fn, arena, short, lens, index, n, pseudo, verify)
    assert err == ERANGE_BIT
    limit = short if unit == 1 else (short + 15) // 16  # the arena's bytes, or its 16-byte chunks
    tiles_ok = [t for t in range((n + 63) // 64) if int(index[t + 1].item()) <= limit]
    assert 0 < len(tiles_ok) < (n + 63) // 64
    for t in range((n + 63) // 64):
        sl = slice(64 * t, min(n, 64 * t + 64))
        if t in tiles_ok:
            assert np.array_equal(got[sl], good[sl]), t
        else:
            assert (got[sl] == 0).all(), t
    # lengths grown after the index was built: the last tile now reaches past the end
    lens2 = lens.clone()
    lens2[n - 1] = -1  # 65535 as u16
    got, err = _run(fn, arena, nbytes, lens2, index, n, pseudo, verify)
    assert err == ERANGE_BIT and (got[64 * 40:] == 0).all()
    assert np.array_equal(got[:64 * 40], good[:64 * 40])
