"""Shared test helpers (parsing of reference fixtures)."""


def curl_desc_and_keys(orc_or_none, ref_fixtures, derive):
    """The curl Initial: long header, DCID 20 B at byte 6; keys from the client initial secret."""
    data = bytes.fromhex(ref_fixtures["curl_initial"]["hex"])
    dcid_len = data[5]
    dcid = data[6:6 + dcid_len]
    pos = 6 + dcid_len
    scid_len = data[pos]
    pos += 1 + scid_len
    tok_len = data[pos]  # 1-byte varint in this capture
    assert tok_len < 64
    pos += 1 + tok_len
    vlen = 1 << (data[pos] >> 6)  # RFC 9000 §16 varint (this capture: 4-byte Length)
    length = int.from_bytes(data[pos:pos + vlen], "big") & ((1 << (8 * vlen - 2)) - 1)
    pn_offset = pos + vlen
    client, _ = derive(dcid)
    return data, dcid, pn_offset, length, client
