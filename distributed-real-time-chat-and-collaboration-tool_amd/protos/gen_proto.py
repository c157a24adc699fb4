"""Emit ``.proto`` files from the schema (``python -m drtc_amd.protos.gen_proto [outdir]``).

The runtime never needs them (descriptors are built in-process, see
registry.py); they are generated for clients in other languages / protoc
users and checked in next to this module.
"""
from __future__ import annotations

import os
import sys

from . import schema


def _ptype(t: str) -> str:
    if t.startswith("."):
        return t[1:]
    return t.replace(",", ", ")


def render(spec: dict) -> str:
    out = ["// GENERATED from drtc_amd/protos/schema.py - do not edit.", 'syntax = "proto3";', "",
           f"package {spec['package']};", ""]
    for imp in spec["imports"]:
        out.append(f'import "{imp}";')
    if spec["imports"]:
        out.append("")
    for sname, methods in spec["services"].items():
        out.append(f"service {sname} {{")
        for name, inp, res, stream in methods:
            out.append(f"  rpc {name}({inp}) returns ({'stream ' if stream else ''}{res});")
        out.append("}")
        out.append("")
    for mname, fields in spec["messages"].items():
        out.append(f"message {mname} {{")
        for fname, num, ftype in fields:
            out.append(f"  {_ptype(ftype)} {fname} = {num};")
        out.append("}")
        out.append("")
    return "\n".join(out)


def main(outdir: str | None = None) -> list[str]:
    outdir = outdir or os.path.dirname(os.path.abspath(__file__))
    os.makedirs(outdir, exist_ok=True)
    paths = []
    for spec in schema.ALL:
        p = os.path.join(outdir, spec["file"])
        with open(p, "w") as f:
            f.write(render(spec))
        paths.append(p)
    return paths


if __name__ == "__main__":
    for p in main(sys.argv[1] if len(sys.argv) > 1 else None):
        print(p)
