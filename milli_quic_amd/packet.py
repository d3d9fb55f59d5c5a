"""Packet-number and header helpers, mirroring src/packet (host side).

These position the AAD, PN and sample for the device batch: ``pn_length`` / ``encode_pn`` /
``decode_pn`` follow src/packet/number.rs:9-70; header builders follow
src/packet/short_header.rs:33-47 and src/packet/long_header.rs:214-314.
"""
MAX_VARINT = (1 << 62) - 1  # src/varint.rs:13
QUIC_VERSION_1 = 1
MIN_INITIAL_PACKET_SIZE = 1200  # src/packet/mod.rs:29


def pn_length(full_pn, largest_acked):
    """number.rs:9-26"""
    num_unacked = full_pn - largest_acked if full_pn > largest_acked else 1
    if num_unacked < (1 << 7):
        return 1
    if num_unacked < (1 << 15):
        return 2
    if num_unacked < (1 << 23):
        return 3
    return 4


def encode_pn(full_pn, largest_acked):
    """number.rs:32-43: the truncated PN in big-endian, pn_length bytes."""
    n = pn_length(full_pn, largest_acked)
    return (full_pn & ((1 << (8 * n)) - 1)).to_bytes(n, "big")


def decode_pn(truncated_pn, pn_len, largest_pn):
    """number.rs:52-70 (RFC 9000 A.3)."""
    pn_nbits = pn_len * 8
    pn_win = 1 << pn_nbits
    pn_hwin = pn_win // 2
    pn_mask = pn_win - 1
    expected_pn = largest_pn + 1
    candidate_pn = (expected_pn & ~pn_mask) | truncated_pn
    if candidate_pn + pn_hwin <= expected_pn and candidate_pn + pn_win <= (1 << 62):
        return candidate_pn + pn_win
    if candidate_pn > expected_pn + pn_hwin and candidate_pn >= pn_win:
        return candidate_pn - pn_win
    return candidate_pn


def encode_varint(v):
    """src/varint.rs encoding (RFC 9000 §16)."""
    if v < 0 or v > MAX_VARINT:
        raise ValueError("varint out of range")
    if v < 1 << 6:
        return bytes([v])
    if v < 1 << 14:
        return (v | 0x4000).to_bytes(2, "big")
    if v < 1 << 30:
        return (v | 0x80000000).to_bytes(4, "big")
    return (v | 0xC000000000000000).to_bytes(8, "big")


def short_header(dcid, pn_len, key_phase=0):
    """First byte 0x40 | kp<<2 | (pn_len-1) (transmit.rs:677-679) followed by the DCID.
    Returns (header_without_pn, pn_offset)."""
    first = 0x40 | ((key_phase & 1) << 2) | ((pn_len - 1) & 3)
    hdr = bytes([first]) + bytes(dcid)
    return hdr, len(hdr)


def initial_header(dcid, scid, token, pn_len, payload_length):
    """encode_initial_header (long_header.rs:214-264). payload_length covers PN + payload + tag."""
    hdr = bytes([0xC0 | ((pn_len - 1) & 3)]) + QUIC_VERSION_1.to_bytes(4, "big")
    hdr += bytes([len(dcid)]) + bytes(dcid) + bytes([len(scid)]) + bytes(scid)
    hdr += encode_varint(len(token)) + bytes(token) + encode_varint(payload_length)
    return hdr, len(hdr)


def handshake_header(dcid, scid, pn_len, payload_length):
    """encode_handshake_header (long_header.rs:271-314)."""
    hdr = bytes([0xE0 | ((pn_len - 1) & 3)]) + QUIC_VERSION_1.to_bytes(4, "big")
    hdr += bytes([len(dcid)]) + bytes(dcid) + bytes([len(scid)]) + bytes(scid)
    hdr += encode_varint(payload_length)
    return hdr, len(hdr)
