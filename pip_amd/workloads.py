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
    description: str = ""

    @property
    def seed(self) -> int:
        return cfg_seed(self.cfg)

    @property
    def ragged(self) -> bool:
        return self.length is None


CFG1 = Workload("cfg1_ipv4_header", 1, 20, HDR_IPV4, 0, 0, 1 << 20, 24,
                "IPv4 20-byte header checksum (pip_ip_checksum), 1M headers")
CFG2 = Workload("cfg2_tcp4_mtu1500", 2, 1480, HDR_TCP, 4, 6, 4 << 20, 1488,
                "TCP/IPv4, 20-B header + 1460-B payload, 4M packets")
CFG3 = Workload("cfg3_udp6_mtu9000", 3, 8960, HDR_UDP, 6, 17, 1 << 20, 8960,
                "UDP/IPv6, 8-B header + 8952-B payload, 1M packets")
CFG4 = Workload("cfg4_tcp4_zipf", 4, None, HDR_TCP, 4, 6, 8 << 20, 0,
                "TCP/IPv4, L4 length 64-9000 B Zipf(1.0), 8M packets (ragged)")
CFG5 = Workload("cfg5_tcp4_mtu9000", 5, 8980, HDR_TCP, 4, 6, 64 << 20, 8992,
                "TCP/IPv4 MTU 9000, 20-B header + 8960-B payload, 64M packets over 8 GPUs")

ALL = {w.name: w for w in (CFG1, CFG2, CFG3, CFG4, CFG5)}
BY_CFG = {w.cfg: w for w in (CFG1, CFG2, CFG3, CFG4, CFG5)}
