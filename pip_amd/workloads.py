"""The five BASELINE.json configurations as data.

Packets are produced on the device by ``pipck_gen_*`` from global packet ids,
so a shard on any GPU holds exactly the bytes the same packet ids hold in a
single-GPU run.  ``first`` is the shard's first global packet id.
"""
from __future__ import annotations

from dataclasses import dataclass

from ._lib import HDR_IPV4, HDR_TCP, HDR_UDP

N_FLOWS = 1024  # 1,024 synthetic (src, dst) pairs, flow = pkt % 1024


def cfg_seed(cfg: int) -> int:
    """0x9E3779B97F4A7C15 ^ cfg (same as pipck_cfg_seed / ock_cfg_seed)."""
    return 0x9E3779B97F4A7C15 ^ cfg


def count_text(n: int) -> str:
    """8388608 -> '8M', 1000 -> '1000' (binary multiples, as BASELINE.json counts packets)."""
    for shift, suffix in ((30, "G"), (20, "M"), (10, "K")):
        if n >= 1 << shift and n % (1 << shift) == 0:
            return f"{n >> shift}{suffix}"
    return f"{n:,}"


@dataclass(frozen=True)
class Workload:
    name: str
    cfg: int
    length: int | None  # L4 bytes checksummed per packet; None = Zipf-ragged
    hdr: int            # header fields the generator writes (th_sum/uh_sum/ip_sum zeroed)
    family: int         # 4 / 6 pseudo-header, 0 = pip_ip_checksum (no pseudo-header)
    proto: int
    n_packets: int      # the BASELINE.json batch (cfg5: the whole 8-GPU job)
    stride: int = 0     # arena slot per packet (fixed configs)
    shape: str = ""     # packet shape, without the count

    @property
    def seed(self) -> int:
        return cfg_seed(self.cfg)

    @property
    def ragged(self) -> bool:
        return self.length is None

    @property
    def description(self) -> str:
        return self.describe(self.n_packets)

    def describe(self, n_packets: int, n_gpus: int = 1) -> str:
        """The workload as run: the packet count is the one actually checksummed."""
        where = f" over {n_gpus} GPUs" if n_gpus > 1 else ""
        return f"{self.shape}, {count_text(n_packets)} packets{where}"


# cfg1 is laid out packed (stride 20 = the header): every fetched byte is a
# header byte, so the launch's HBM traffic is the algorithmic 22 B per header.
CFG1 = Workload("cfg1_ipv4_header", 1, 20, HDR_IPV4, 0, 0, 1 << 20, 20,
                "IPv4 20-byte header checksum (pip_ip_checksum), packed 20-B stride")
CFG2 = Workload("cfg2_tcp4_mtu1500", 2, 1480, HDR_TCP, 4, 6, 4 << 20, 1488,
                "TCP/IPv4, 20-B header + 1460-B payload")
CFG3 = Workload("cfg3_udp6_mtu9000", 3, 8960, HDR_UDP, 6, 17, 1 << 20, 8960,
                "UDP/IPv6, 8-B header + 8952-B payload")
CFG4 = Workload("cfg4_tcp4_zipf", 4, None, HDR_TCP, 4, 6, 8 << 20, 0,
                "TCP/IPv4, L4 length 64-9000 B Zipf(1.0), ragged")
CFG5 = Workload("cfg5_tcp4_mtu9000", 5, 8980, HDR_TCP, 4, 6, 64 << 20, 8992,
                "TCP/IPv4 MTU 9000, 20-B header + 8960-B payload")

ALL = {w.name: w for w in (CFG1, CFG2, CFG3, CFG4, CFG5)}
BY_CFG = {w.cfg: w for w in (CFG1, CFG2, CFG3, CFG4, CFG5)}
