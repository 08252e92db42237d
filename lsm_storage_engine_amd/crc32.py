"""crc::crc32 stand-in: the scalar CRC-32/ISO-HDLC entry points.

Mirrors the one function of crate `crc` ^1.7 the reference uses,
``crc::crc32::checksum_ieee(&[u8]) -> u32`` (src/wal.rs:135,153,177,187),
through liblsmck's scalar CPU path (lsmck_crc32_ieee).  Bulk checksumming goes
through ``device.Context.crc32*`` (GPU).
"""
from . import _lib


def checksum_ieee(data) -> int:
    """crc::crc32::checksum_ieee: CRC-32/ISO-HDLC of ``data``."""
    b = bytes(data)
    return _lib.load().lsmck_crc32_ieee(b, len(b))


def update(crc: int, data) -> int:
    """CRC of A||B from crc(A) and the bytes of B (zlib crc32 convention)."""
    b = bytes(data)
    return _lib.load().lsmck_crc32_update(crc & 0xFFFFFFFF, b, len(b))


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """CRC of A||B from crc(A), crc(B) and len(B)."""
    return _lib.load().lsmck_crc32_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)
