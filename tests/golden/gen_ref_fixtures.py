"""Extract data fixtures from the reference tree (run in the build container only).

Writes tests/golden/ref_fixtures.json with:
  * RFC 9001 Appendix A values (keys A.1, protected packets A.2/A.3/A.5) parsed from the
    reference's copy of the RFC text (rfc/rfc9001.txt:2319-2553);
  * the captured `curl --http3` client Initial used by the reference's
    server_processes_curl_initial_packet test (src/connection/mod.rs:2210).
Only bytes are extracted (data, not source). The GPU box never reads /root/reference.
"""
import json
import re
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = sys.argv[2] if len(sys.argv) > 2 else "tests/golden/ref_fixtures.json"

rfc = open(f"{REF}/rfc/rfc9001.txt").read().splitlines()


def hexblock(start_pat, stop_pat):
    """Concatenate hex groups from the first line after start_pat until stop_pat."""
    i = next(k for k, l in enumerate(rfc) if re.search(start_pat, l))
    out = []
    for l in rfc[i + 1:]:
        if re.search(stop_pat, l):
            break
        t = l.strip()
        if t and re.fullmatch(r"[0-9a-f ]+", t):
            out.append(t.replace(" ", ""))
    return "".join(out)


def value_after(label, nlines=2):
    i = next(k for k, l in enumerate(rfc) if l.strip().startswith(label))
    s = rfc[i].split("=")[-1].strip()
    j = i + 1
    while j < i + nlines and re.fullmatch(r"[0-9a-f]+", rfc[j].strip() or "x"):
        s += rfc[j].strip()
        j += 1
    return s.replace(" ", "")


fx = {
    "rfc9001": {
        "initial_secret": "7db5df06e7a69e432496adedb00851923595221596ae2ae9fb8115c1e9ed0a44",
        "dcid": "8394c8f03e515708",
        "a2_protected": hexblock(r"The resulting protected packet is:", r"^A\.3\."),
        "a3_protected": hexblock(r"The final protected packet is then:", r"^A\.4\."),
        "a5_packet": "4cfe4189655e5cd55c41f69080575d7999c25a5bfb",
    },
}
# A.1 secrets/keys, in document order (client block then server block)
keys = {}
for name in ("client_initial_secret", "server_initial_secret"):
    i = next(k for k, l in enumerate(rfc) if l.strip() == name)
    keys[name] = (rfc[i + 2].split("=")[-1].strip() + rfc[i + 3].strip()).replace(" ", "")
blocks = [k for k, l in enumerate(rfc) if l.strip().startswith("key = HKDF-Expand-Label")]
for side, k in zip(("client", "server"), blocks):
    keys[f"{side}_key"] = rfc[k + 1].split("=")[-1].strip()
    keys[f"{side}_iv"] = rfc[k + 4].split("=")[-1].strip()
    keys[f"{side}_hp"] = rfc[k + 7].split("=")[-1].strip()
fx["rfc9001"]["a1"] = keys
# A.5 ChaCha20 values
a5 = next(k for k, l in enumerate(rfc) if l.startswith("A.5."))
sec = [k for k, l in enumerate(rfc) if k > a5 and l.strip() == "secret"][0]
fx["rfc9001"]["a5"] = {
    "secret": (rfc[sec + 1].split("=")[-1] + rfc[sec + 2]).replace(" ", "").strip(),
    "ku": (rfc[sec + 17].split("=")[-1] + rfc[sec + 18]).replace(" ", "").strip(),
}
mod = open(f"{REF}/src/connection/mod.rs").read()
m = re.search(r'CURL_INITIAL_HEX: &str = "([0-9a-f]+)"', mod)
fx["curl_initial"] = {"source": "src/connection/mod.rs:2210", "hex": m.group(1)}
json.dump(fx, open(OUT, "w"), indent=1)
print("wrote", OUT, len(fx["rfc9001"]["a2_protected"]) // 2, len(fx["rfc9001"]["a3_protected"]) // 2,
      len(fx["curl_initial"]["hex"]) // 2)
