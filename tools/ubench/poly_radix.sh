#!/bin/bash
# Poly1305 step radix comparison: CPU check of the three forms, then VALU counts of
# each kernel's lean loop from the gfx950 assembly. No GPU needed. Output: stdout.
set -euo pipefail
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 poly_radix.hip -o /tmp/poly_radix
/tmp/poly_radix > /tmp/poly_radix.out
python3 - <<'PY'
P = (1 << 130) - 5
bad = n = 0
for line in open("/tmp/poly_radix.out"):
    f = line.split()
    if f[0] == "T" and f[1] == "r":
        r = sum(int(x) << (32 * i) for i, x in enumerate(f[2:])); hr = hg = 0
    elif f[0] == "T" and f[1] == "g":
        g = sum(int(x) << (32 * i) for i, x in enumerate(f[2:]))
    elif f[0] == "B":
        m = sum(int(x) << (32 * i) for i, x in enumerate(f[1:])) + (1 << 128)
        hr = (hr + m) * r % P; hg = (hg + m) * g % P
    elif f[0] == "H":
        w = [int(x) for x in f[2:]]
        v = sum(x << (26 * i) for i, x in enumerate(w)) if f[1].startswith("p26") else sum(x << (32 * i) for i, x in enumerate(w))
        want = hg if f[1].endswith("g") else hr
        n += 1; bad += (v % P) != want
print(f"cpu check against Python ints: {bad} mismatches of {n} (200 trials x 40 blocks x 4 forms)")
PY
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S poly_radix.hip -o /tmp/poly_radix.s
python3 - <<'PY'
import re
s = open("/tmp/poly_radix.s").read().split("\n")
for name in ("p26", "p32c", "p32g"):
    a = next(i for i, l in enumerate(s) if f"LOOP_START {name}" in l)
    b = next(i for i, l in enumerate(s) if f"LOOP_END {name}" in l)
    body = [l.strip() for l in s[a:b] if l.strip() and not l.strip().startswith((";", ".", "s_cbranch")) and not l.strip().endswith(":")]
    v = [l for l in body if l.startswith("v_")]
    mad = [l for l in v if l.startswith("v_mad_u64_u32")]
    mem = [l for l in body if l.startswith(("global_", "buffer_", "flat_"))]
    print(f"{name:5s} VALU per step {len(v):3d} (v_mad_u64_u32 {len(mad)}), memory {len(mem)}, all {len(body)}")
PY
