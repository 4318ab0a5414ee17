"""pip_amd -- MI355X-native Internet-checksum engine for plumk97/pip's checksum path.

Layout:
  csrc/          HIP kernels for gfx950 + the C ABI (include/pipck.h) + the C++
                 drop-in for pip's six functions (include/pip_checksum_amd.h)
  lib/           in-tree build output (libpipck.so, libpip_checksum_amd.so)
  engine.py      device-resident batch calls (torch tensors as memory/streams)
  checksum.py    pip's per-packet API, same names, on the GPU
  workloads.py   the BASELINE.json configurations
  shard.py       packet-range sharding across GPUs (no collectives on the data path)
"""
from ._lib import LIB_DIR, LIBPIPCK, LIBSHIM, PipckError, load  # noqa: F401

__version__ = "0.1.0"
