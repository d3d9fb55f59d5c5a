"""Extract TLS 1.3 record-protection vectors from the reference tree (build container only).

Writes tests/golden/tls_records.json: the AES-128-GCM records of RFC 8448 §3 ("Simple 1-RTT
Handshake") as shipped in the reference's copy of the RFC (rfc/rfc8448.txt:360-855): for each
record the write key / iv of its direction and epoch, its sequence number, the inner content
type, the plaintext payload and the complete protected record. They pin the record layer of the
reference (src/tcp_tls/record.rs:70-143, src/tcp_tls/connection.rs:546-600). Only bytes are
extracted (data, not source). The GPU box never reads /root/reference.
"""
import json
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = sys.argv[2] if len(sys.argv) > 2 else "tests/golden/tls_records.json"

lines = open(f"{REF}/rfc/rfc8448.txt").read().split("\n")  # not splitlines(): keep form feeds in-line
END = next(k for k, l in enumerate(lines) if l.startswith("4.  Resumed 0-RTT Handshake"))


def hex_after(i):
    """Octets of the labelled value on line i; continuation lines are pure hex, page breaks
    between them are skipped."""
    n = int(re.search(r"\((\d+) octets\)", lines[i]).group(1))
    octets = lines[i].split(":", 1)[1].split()
    j = i + 1
    while len(octets) < n:
        t = lines[j].strip()
        if re.fullmatch(r"([0-9a-f]{2} ?)+", t):
            octets += t.split()
        j += 1
    assert len(octets) == n, (i, len(octets), n)
    return "".join(octets)


def find(pat, start=0):
    return next(k for k in range(start, END) if re.search(pat, lines[k]))


def keys(block_pat):
    b = find(block_pat)
    return hex_after(find(r"key expanded", b)), hex_after(find(r"iv expanded", b))


server_hs = keys(r"\{server\}  derive write traffic keys for handshake data")
client_hs = keys(r"\{server\}  derive read traffic keys for handshake data")  # = client write
server_ap = keys(r"\{server\}  derive write traffic keys for application data")
client_ap = keys(r"\{client\}  derive write traffic keys for application data")

# (sender block, occurrence, write keys, sequence number, inner content type)
plan = [
    (r"\{server\}  send handshake record", 1, server_hs, 0, 0x16),  # EE..Finished (occ. 0: ServerHello)
    (r"\{client\}  send handshake record", 1, client_hs, 0, 0x16),  # Finished (occ. 0: ClientHello)
    (r"\{server\}  send handshake record", 2, server_ap, 0, 0x16),  # NewSessionTicket
    (r"\{client\}  send application_data record", 0, client_ap, 0, 0x17),
    (r"\{server\}  send application_data record", 0, server_ap, 1, 0x17),
    (r"\{client\}  send alert record", 0, client_ap, 1, 0x15),
    (r"\{server\}  send alert record", 0, server_ap, 2, 0x15),
]
recs = []
for pat, occ, (key, iv), seq, ctype in plan:
    s = [k for k in range(END) if re.search(pat, lines[k])][occ]
    recs.append({"source": f"rfc/rfc8448.txt:{s + 1}", "suite": 1, "key": key, "iv": iv, "seq": seq,
                 "inner_type": ctype, "payload": hex_after(find(r"payload \(", s)),
                 "record": hex_after(find(r"complete record \(", s))})
json.dump({"source": "RFC 8448 §3 (reference rfc/rfc8448.txt), TLS_AES_128_GCM_SHA256", "records": recs},
          open(OUT, "w"), indent=1)
print("wrote", OUT, [len(r["record"]) // 2 for r in recs])
