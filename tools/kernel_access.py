#!/usr/bin/env python3
"""Static field-access map of the dycore's HIP kernels: for every __global__ kernel, the Ptrs
fields (and pointer arguments) it reads and writes, following the __device__ helpers it calls.

Used by tools/kernel_roofline.py to count algorithmic bytes per launch (each
distinct array read once and / or written once per call).  Writes are `p.X[..] = ...`,
`st2(p.X + ...)` and stores through a pointer argument; every other mention is a read.  It is a
text scan, so it reports what a kernel *may* touch: branches the launch parameters switch off
(rk_step, store flags, physics) are resolved by the per-kernel rules in kernel_roofline.py.

    python tools/kernel_access.py [kernel-name-substring]
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "mpas-model_amd", "csrc")
FILES = ["kernels.hip", "lbc.hip", "summary.hip", "halo.hip"]


def _bodies(text):
    """name -> (kind, signature, body) for every __global__ / __device__ function."""
    out = {}
    for m in re.finditer(r"(__global__|__device__)[^;{]*?\b(\w+)\s*\(", text):
        kind, name = m.group(1), m.group(2)
        depth, j = 1, m.end()  # the closing parenthesis of the parameter list
        while j < len(text) and depth:
            depth += {"(": 1, ")": -1}.get(text[j], 0)
            j += 1
        i = text.find("{", j)
        semi = text.find(";", j)
        if i < 0 or (0 <= semi < i):
            continue
        sig = text[m.start():i]
        depth, j = 0, i
        while j < len(text):
            if text[j] == "{":
                depth += 1
            elif text[j] == "}":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        out.setdefault(name, []).append((kind, sig, text[i:j + 1]))
    return out


def _strip_comments(s):
    s = re.sub(r"//[^\n]*", "", s)
    s = re.sub(r"__launch_bounds__\([^)]*\)", "", s)
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def access_map():
    text = "".join(_strip_comments(open(os.path.join(CSRC, f)).read()) for f in FILES
                   if os.path.isfile(os.path.join(CSRC, f)))
    bodies = _bodies(text)
    helpers = {n: v for n, v in bodies.items() if any(k == "__device__" for k, _, _ in v)}

    def scan(body, seen):
        reads, writes = set(), set()
        for m in re.finditer(r"\bp\.(\w+)", body):
            f = m.group(1)
            after = body[m.end():m.end() + 200]
            before = body[max(0, m.start() - 12):m.start()]
            w = False
            if re.match(r"\s*\[[^\]]*\]\s*=[^=]", after) or re.match(r"\s*\[[^\]]*\]\s*(\+|-|\*)=", after):
                w = True
            if re.search(r"(st2|store|pack_column|atomicAdd)\(\s*$", before):
                w = True
            (writes if w else reads).add(f)
        for name, defs in helpers.items():
            if name in seen or not re.search(rf"\b{name}\s*[<(]", body):
                continue
            for _, _, hb in defs:
                r, w = scan(hb, seen | {name})
                reads |= r
                writes |= w
        return reads, writes

    out = {}
    for name, defs in bodies.items():
        for kind, sig, body in defs:
            if kind != "__global__":
                continue
            r, w = scan(body, {name})
            out[name] = (sorted(r - {"cf1", "cf2", "cf3"}), sorted(w))
    return out


if __name__ == "__main__":
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    for k, (r, w) in sorted(access_map().items()):
        if pat in k:
            print(f"{k}\n  R: {' '.join(r)}\n  W: {' '.join(w)}")
