"""AddressSanitizer build of the C-ABI's host code and its argument-validation check (SURVEY.md §5:
"run the C++ host code under ASan in the CPU-only build").

  python tools/asan_abi.py [--out DIR]      build (if stale) and run; exit 0 when every case passes

1. Every csrc/*.hip is compiled with `-Xarch_host -fsanitize=address` (host code instrumented;
   the device code is built as usual and never runs here) into DIR/libregcn_hip_asan.so.
2. A C++ harness is generated from include/regcn_hip.h (every prototype, so a new export is
   covered without editing this file) and linked with -fsanitize=address against that library.
   Its cases, each of which must return a negative REGCN_E* code with an error string set:
   * null:      every pointer argument NULL, every size 64 (the stream NULL = default stream);
   * zero desc: descriptor-taking exports with an all-zero descriptor;
   * bad d:     d = -4 with non-null pointers; d = 1000 where the export documents d <= 256;
   * odd d:     the Givens rotation (the ABI takes interleaved pairs: an odd row width shows
                as pairs off 8-byte alignment) and a negative pair count;
   * workspace: the order / transpose / snapshot builders with ws_bytes = 1, and the CE with a
                NULL workspace.
   Size queries (the *_bytes / *_floats / capacity exports) are called for crashes only.
   The harness runs with ASAN_OPTIONS=detect_leaks=0 (the HIP runtime's own allocations) and
   no GPU: a case that slipped past validation would reach a HIP call, which returns a
   positive hipError_t here and is reported as a failure.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "re-gcn_amd", "csrc")
HEADER = os.path.join(REPO, "include", "regcn_hip.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ASAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-fPIC", "-ffp-contract=on", "-Wno-unused-function"]

# exports documented to take d <= 256 (fixed register / LDS tiles)
# (the scorer itself takes any d % 4 == 0: d > 256 runs its general kernel)
D_MAX_256 = ("regcn_layer_tail_f32", "regcn_timestep_f32", "regcn_timestep_analysis_f32",
             "regcn_hyp_ce_bwd_f32", "regcn_rowmap_bwd_f32",
             "regcn_relation_gru_f32", "regcn_relation_gru_pre_f32", "regcn_relation_gru_x_f32",
             "regcn_roth_query_f32", "regcn_roth_rel_query_f32", "regcn_lorentz_centroid_f32")
NOT_INT = ("regcn_version", "regcn_set_trace", "regcn_last_error_string")


def prototypes():
    s = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = []
    for ret, name, args in re.findall(r"^\s*([A-Za-z_][\w\s\*]*?)\b(regcn_\w+)\s*\(([^;{]*?)\)\s*;", s, flags=re.M):
        params = []
        for a in args.split(","):
            a = " ".join(a.split())
            if not a or a == "void":
                continue
            m = re.match(r"(.*?)(\w+)$", a)
            params.append((m.group(1).strip(), m.group(2)))
        out.append((ret.strip(), name, params))
    return out


def _arg(t, n, mode, override):
    if n in override:
        return override[n]
    if "*" in t:
        if mode == "null" or n == "stream":
            return "nullptr"
        return "(%s)dummy" % t
    if t == "float":
        return "0.01f"
    if t == "size_t":
        return "(size_t)1 << 20"
    return "64"


def harness():
    lines = ['#include <stdio.h>', '#include <string.h>', '#include "regcn_hip.h"',
             "static unsigned char dummy_buf[1 << 20] __attribute__((aligned(256)));",
             "static void* dummy = dummy_buf;", "static int fails = 0, cases = 0;",
             "static void expect_neg(int rc, const char* what) {",
             "  cases++;",
             "  const char* e = regcn_last_error_string();",
             "  if (rc >= 0 || !e || !e[0]) { printf(\"FAIL %s: rc=%d err='%s'\\n\", what, rc, e ? e : \"\"); fails++; }",
             "}", "int main() {"]
    for ret, name, params in prototypes():
        call = lambda mode, ov=None: "%s(%s)" % (name, ", ".join(_arg(t, n, mode, ov or {}) for t, n in params))
        if name in NOT_INT or ret != "int":
            lines.append("  (void)%s;" % call("null"))
            continue
        lines.append('  expect_neg(%s, "%s null");' % (call("null"), name))
        descs = [(t, n) for t, n in params if "regcn_" in t and "*" in t]
        for t, n in descs:
            base = t.replace("const", "").replace("*", "").strip()
            ov = {n: "z_%s" % n}
            lines.append("  { static %s z_%s[4]; memset(z_%s, 0, sizeof(z_%s));" % (base, n, n, n))
            lines.append('    expect_neg(%s, "%s zero desc"); }' % (call("null", ov), name))
        names = [n for _, n in params]
        if "d" in names and not descs:
            lines.append('  expect_neg(%s, "%s d=-4");' % (call("dummy", {"d": "-4"}), name))
            if name in D_MAX_256:
                lines.append('  expect_neg(%s, "%s d=1000");' % (call("dummy", {"d": "1000"}), name))
        if name == "regcn_givens_rotation_f32":  # the ABI takes pairs: an odd row width shows as
            # a pair straddling 8-byte alignment (x + 1 float) or a negative pair count
            lines.append('  expect_neg(%s, "%s odd d (misaligned pairs)");'
                         % (call("dummy", {"x": "(const float*)dummy + 1"}), name))
            lines.append('  expect_neg(%s, "%s n_pairs=-2");' % (call("dummy", {"n_pairs": "-2"}), name))
        if "ws_bytes" in names:
            lines.append('  expect_neg(%s, "%s ws_bytes=1");' % (call("dummy", {"ws_bytes": "1"}), name))
        if name in ("regcn_hyp_ce_f32", "regcn_hyp_ce_lse_f32"):
            lines.append('  expect_neg(%s, "%s null workspace");' % (call("dummy", {"workspace": "nullptr"}), name))
    # descriptors with every buffer set but an undersized workspace
    lines += [
        "  { regcn_snapshot_desc s; memset(&s, 0, sizeof(s));",
        "    void** p = (void**)&s; (void)p;",
        "    s.triples = (const int64_t*)dummy; s.T = 64; s.V = 64; s.R = 8; s.budget = 4096; s.pack_items = 1;",
        "    s.chunk_edges = 1024; s.workspace = dummy; s.ws_bytes = 1; s.stats = (int32_t*)dummy;",
        "    s.in_deg = s.rowptr = s.col_src = s.col_type = s.rel_ent_count = s.rel_idx = s.rel_start = (int32_t*)dummy;",
        "    s.norm = s.edge_norm = s.rel_count = (float*)dummy; s.edge_type = (int64_t*)dummy;",
        "    s.rows = s.tiles = s.item_ptr = s.item_src = s.item_tl = s.chunks = s.fixups = (int32_t*)dummy;",
        "    s.heavy_chunks = s.heavy_fixups = s.rel_chunks = s.rel_fixups = (int32_t*)dummy;",
        '    expect_neg(regcn_snapshot_csr_i32(&s, nullptr), "regcn_snapshot_csr_i32 ws_bytes=1");',
        '    expect_neg(regcn_snapshot_work_i32(&s, nullptr), "regcn_snapshot_work_i32 ws_bytes=1"); }',
        "  { regcn_transpose_desc t; memset(&t, 0, sizeof(t)); t.V = 64; t.E = 64; t.R2 = 8;",
        "    t.rowptr = t.col_src = t.col_type = (const int32_t*)dummy; t.workspace = dummy; t.ws_bytes = 1;",
        "    t.csr_dst = t.sptr = t.sp = t.tptr = t.tp = (int32_t*)dummy;",
        '    expect_neg(regcn_snapshot_transpose_i32(&t, nullptr), "regcn_snapshot_transpose_i32 ws_bytes=1"); }',
        '  printf("asan abi check: %d cases, %d failed\\n", cases, fails);',
        "  return fails ? 1 : 0;", "}"]
    return "\n".join(lines) + "\n"


def _stale(out, deps):
    return not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(p) for p in deps)


def build(out_dir):
    os.makedirs(out_dir, exist_ok=True)
    sys.path.insert(0, REPO)
    from __graft_entry__ import SOURCES
    headers = glob.glob(os.path.join(CSRC, "*.h")) + [HEADER]

    def comp(src):
        obj = os.path.join(out_dir, src.replace(".hip", ".o"))
        if _stale(obj, [os.path.join(CSRC, src)] + headers):
            subprocess.run([HIPCC, *FLAGS, *ASAN, "-I", os.path.join(REPO, "include"), "-c",
                            os.path.join(CSRC, src), "-o", obj], check=True)
        return obj
    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, SOURCES))
    lib = os.path.join(out_dir, "libregcn_hip_asan.so")
    if _stale(lib, objs):
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *ASAN, "-o", lib, *objs], check=True)
    src = os.path.join(out_dir, "abi_check.cpp")
    text = harness()
    if not os.path.exists(src) or open(src).read() != text:
        with open(src, "w") as f:
            f.write(text)
    exe = os.path.join(out_dir, "abi_check")
    if _stale(exe, [src, lib, HEADER]):
        subprocess.run(["/opt/rocm/llvm/bin/clang++", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                        "-I", os.path.join(REPO, "include"), src, "-o", exe, "-L", out_dir, "-lregcn_hip_asan",
                        "-Wl,-rpath," + out_dir, "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"],
                       check=True)
    return exe


def run(exe):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", HIP_VISIBLE_DEVICES="-1",
               ROCR_VISIBLE_DEVICES="-1")
    return subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(CSRC, "build", "asan"))
    a = ap.parse_args()
    r = run(build(a.out))
    sys.stdout.write(r.stdout)
    sys.stderr.write(r.stderr[-4000:])
    sys.exit(r.returncode)


if __name__ == "__main__":
    main()
