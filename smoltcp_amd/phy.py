"""Checksum policy, mirroring ``smoltcp::phy::{Checksum, ChecksumCapabilities}``
(src/phy/mod.rs:173-234)."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field


class Checksum(enum.IntEnum):
    """phy::Checksum (src/phy/mod.rs:176-186); ``Both`` is the default (:178)."""

    Both = 0
    Rx = 1
    Tx = 2
    None_ = 3

    def rx(self) -> bool:  # src/phy/mod.rs:188-194
        return self in (Checksum.Both, Checksum.Rx)

    def tx(self) -> bool:  # src/phy/mod.rs:196-203
        return self in (Checksum.Both, Checksum.Tx)


@dataclass
class ChecksumCapabilities:
    """phy::ChecksumCapabilities (src/phy/mod.rs:210-218)."""

    ipv4: Checksum = field(default=Checksum.Both)
    udp: Checksum = field(default=Checksum.Both)
    tcp: Checksum = field(default=Checksum.Both)
    icmpv4: Checksum = field(default=Checksum.Both)
    icmpv6: Checksum = field(default=Checksum.Both)

    @staticmethod
    def ignored() -> "ChecksumCapabilities":  # src/phy/mod.rs:223-233
        n = Checksum.None_
        return ChecksumCapabilities(n, n, n, n, n)

    def as_tuple(self):
        return (int(self.ipv4), int(self.udp), int(self.tcp), int(self.icmpv4), int(self.icmpv6))
