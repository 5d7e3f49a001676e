"""A/B build of libregcn_hip.so with per-source extra flags (the _lib loader takes the variant via
REGCN_HIP_LIB).  Objects of the unchanged sources are the default build's.

  python tools/build_variant.py --name w8 --src timestep.hip --flags -DREGCN_ROWTILE_WAVES=8
  -> re-gcn_amd/regcn_amd/libregcn_hip_w8.so
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", required=True)
    ap.add_argument("--src", required=True, help="comma-separated sources built with the extra flags")
    ap.add_argument("--flags", nargs=argparse.REMAINDER, default=[])
    a = ap.parse_args()
    G.build()
    out_dir = os.path.join(G.CSRC, "build", a.name)
    os.makedirs(out_dir, exist_ok=True)
    special = set(a.src.split(","))
    objs = []
    for src in G.SOURCES:
        if src in special:
            obj = os.path.join(out_dir, src.replace(".hip", ".o"))
            subprocess.run([G.HIPCC, *G.FLAGS, *G.SOURCE_FLAGS.get(src, []), *a.flags, "-c", os.path.join(G.CSRC, src), "-o", obj], check=True)
        else:
            obj = os.path.join(G.CSRC, "build", src.replace(".hip", ".o"))
        objs.append(obj)
    lib = os.path.join(os.path.dirname(G.LIB), "libregcn_hip_%s.so" % a.name)
    subprocess.run([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
