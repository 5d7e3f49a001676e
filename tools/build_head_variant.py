"""A/B helper: link libregcn_hip_<name>.so from the current objects but with the listed sources
compiled from git HEAD (the committed version), so one GPU run can time both builds.

  python tools/build_head_variant.py --name head --src rowtail.hip,score.hip
"""
import argparse
import os
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", required=True)
    ap.add_argument("--src", required=True)
    a = ap.parse_args()
    G.build()
    special = set(a.src.split(","))
    tmp = tempfile.mkdtemp()
    inc = os.path.join(tmp, "include")
    src_dir = os.path.join(tmp, "re-gcn_amd", "csrc")
    os.makedirs(inc)
    os.makedirs(src_dir)
    for f in os.listdir(G.CSRC):
        if f.endswith(".h"):
            with open(os.path.join(src_dir, f), "w") as o:
                o.write(subprocess.run(["git", "show", "HEAD:re-gcn_amd/csrc/" + f], cwd=REPO, check=True,
                                       capture_output=True, text=True).stdout)
    with open(os.path.join(inc, "regcn_hip.h"), "w") as o:
        o.write(subprocess.run(["git", "show", "HEAD:include/regcn_hip.h"], cwd=REPO, check=True,
                               capture_output=True, text=True).stdout)
    objs = []
    for src in G.SOURCES:
        if src in special:
            p = os.path.join(src_dir, src)
            with open(p, "w") as o:
                o.write(subprocess.run(["git", "show", "HEAD:re-gcn_amd/csrc/" + src], cwd=REPO, check=True,
                                       capture_output=True, text=True).stdout)
            obj = os.path.join(tmp, src.replace(".hip", ".o"))
            subprocess.run([G.HIPCC, *G.FLAGS, *G.SOURCE_FLAGS.get(src, []), "-c", p, "-o", obj], check=True)
        else:
            obj = os.path.join(G.CSRC, "build", src.replace(".hip", ".o"))
        objs.append(obj)
    lib = os.path.join(os.path.dirname(G.LIB), "libregcn_hip_%s.so" % a.name)
    subprocess.run([G.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib, *objs], check=True)
    print(lib)


if __name__ == "__main__":
    main()
