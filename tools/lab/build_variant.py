"""Build an A/B variant of libpk_kernels from a patched COPY of csrc/kernels (the production sources
stay free of lab switches).  A variant is a list of (file, old, new) text replacements; the result
lands in tools/lab/libpk_kernels_<variant>.so and is loaded instead of the in-tree library with
POLYKEY_LIB_LIBPK_KERNELS=<path> (polykey_service_amd/_native/loader.py).

    python tools/lab/build_variant.py pre0 mlp_nt
"""
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from polykey_service_amd._native.build import HIP_FLAGS, HIPCC  # noqa: E402

VARIANTS = {
    # round 5, measured and removed: "push_nofence" / "push_nostore" (the TP push epilogue without
    # its system release / without its stores: the release was 3.2 us of the 6.5 us the epilogue
    # added to the 70B TP=8 o projection, the stores 1.1 us -- profiles/r5_push_probe.jsonl; the
    # epilogue now stores write-through at system scope and stamps the flag without a fence)
    # the fused QKV -> attention launch without the K/V prefetch before the hand-off wait
    "pre0": [("decode_fused.hip", "decode_tile<P, kDecodeWaves, true, SS, 2, 2>(",
              "decode_tile<P, kDecodeWaves, true, SS, 2, 0>(")],
    # the fused MLP's down tiles with non-temporal weight loads
    "mlp_nt": [("gemm_skinny.hip", "mlp_fused_kernel<MT, KR><<<", "mlp_fused_kernel<MT, KR, true><<<")],
    # the fused launches' hand-off pollers sleeping 4 instead of 16 (x 64 cycles) between polls
    "sleep4": [("flow.h", "__builtin_amdgcn_s_sleep(16);", "__builtin_amdgcn_s_sleep(4);")],
    # ablations of the 4-wave prefill GEMM measured this round (timing only, wrong results;
    # profiles/r4_prefill_gemm_4wave.md): no LDS-DMA in the k-loop ("pg_noglds", 1,172 vs 1,552 us
    # at gate_up), A loads only ("pg_aonly", 1,287 vs 1,497), no vmcnt waits ("pg_novm", no change),
    # no fragment reads ("pg_nords", -7 %), no barrier ("pg_nobar", no change), full 128-byte lines
    # per row ("pg_fullline", -5.6 %)
    # the 4-wave prefill GEMM's 16 LDS-DMA loads of a tile, measured at gate_up against 2 per group
    # (1,453 us): all right after the barrier ("pg_front") 1,535, 4 per group in the first 4 groups
    # ("pg_first4") 1,443 (noise) -- profiles/r4_prefill_gemm_4wave.md
    # round 6 ablations of the 4-wave prefill GEMM's buffer_load ... lds staging (timing only, wrong
    # results; profiles/r6_prefill_gemm_buffer_lds.md): no vmcnt wait before the tile barrier
    # (gate_up 1,350 vs 1,393 us), no loads in the k-loop (1,151: 7 % under hipBLASLt)
    "pb_novm": [("gemm_prefill.hip", "if constexpr (BAR) wait_vm<0>();", "")],
    "pb_noload": [("gemm_prefill.hip", "if constexpr (LOAD) stage_one(2 * mf, (u + 3) >> 1);", ""),
                  ("gemm_prefill.hip", "if constexpr (LOAD) stage_one(2 * mf + 1, (u + 3) >> 1);", "")],
    # cache policy of the prefill GEMM's staging loads: sc0 (aux 1) on the W / A stream, nt (aux 2) on W
    "pb_sc0_w": [("gemm_prefill.hip", "wvo[j - 8], wo, 0, 0);", "wvo[j - 8], wo, 0, 1);")],
    "pb_sc0_a": [("gemm_prefill.hip", "avo[j], static_cast<unsigned>(T) * BK * 2u, 0, 0);",
                  "avo[j], static_cast<unsigned>(T) * BK * 2u, 0, 1);")],
    "pb_nt_w": [("gemm_prefill.hip", "wvo[j - 8], wo, 0, 0);", "wvo[j - 8], wo, 0, 2);")],
    "pb_split": [("gemm_prefill.hip", "constexpr bool kSplitLoads = false;", "constexpr bool kSplitLoads = true;")],
    # the 4-wave prefill GEMM without the XOR chunk swizzle (lanes of a row in natural order: whole
    # 64-byte lane groups for the address unit, LDS bank conflicts on the fragment reads instead)
    "pb_noswz": [("gemm_prefill.hip", "const int logical = (tid & 7) ^ ((tid >> 4) & 7);", "const int logical = tid & 7;"),
                 ("gemm_prefill.hip", "auto a_off = [&](int s) { return (wr * 128 + r) * BK + (((4 * s + g) ^ ((r >> 1) & 7)) * 8); };",
                  "auto a_off = [&](int s) { return (wr * 128 + r) * BK + ((4 * s + g) * 8); };"),
                 ("gemm_prefill.hip", "    return (wc * 128 + r) * BK + (((4 * s + g) ^ ((r >> 1) & 7)) * 8);",
                  "    return (wc * 128 + r) * BK + ((4 * s + g) * 8);")],
    # round 5, measured and removed: "mt8_chunk256" (128-row decode tiles staging A per 256-deep chunk,
    # one workgroup per CU: 8B at 128 rows 6.36 vs 5.62-5.65 ms, 256 rows 10.07-10.09 vs 9.21-9.22,
    # profiles/r5_mt8.jsonl); "wdepth4" (decode GEMM tiles with four 128-deep weight k-steps
    # in flight per wave instead of two: 8B step 4.22-4.23 vs 3.99-4.00 ms, 70B TP=8 rank 6.77 vs
    # 6.54-6.57 -- profiles/r5_wdepth.jsonl)
    # measured and removed this round (variant builds of the sources of that time): "mlp_v0" (no NT /
    # LDS prefetch in the down tiles: 4.063 vs 4.063 ms per graph-captured 8B step), "o_ring2" (the
    # o-projection without whole-slice weight registers: 3.997 vs 4.063 ms) -- profiles/r4_variant_ab.jsonl
}


# variants of libpk_comm (csrc/comm), loaded with POLYKEY_LIB_LIBPK_COMM=<path>
COMM_VARIANTS = {
    # timing only (NOT coherent): the collectives without their system-scope release / acquire
    # fences (tools/car_probe.py on a loopback group)
    "car_norel": [("custom_allreduce.hip", '__builtin_amdgcn_fence(__ATOMIC_RELEASE, "");', "")],
    "car_noacq": [("custom_allreduce.hip", '__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");', "")],
}


def build_comm(name: str) -> str:
    work = tempfile.mkdtemp(prefix=f"pkvar_{name}_")
    cdir = os.path.join(work, "comm")
    shutil.copytree(os.path.join(REPO, "csrc", "comm"), cdir)
    for fname, old, new in COMM_VARIANTS[name]:
        p = os.path.join(cdir, fname)
        text = open(p).read()
        if old not in text:
            raise SystemExit(f"variant {name}: pattern not found in {fname}: {old!r}")
        open(p, "w").write(text.replace(old, new))
    objs = []
    for s in sorted(glob.glob(os.path.join(cdir, "*.hip"))):
        o = os.path.join(work, os.path.basename(s) + ".o")
        subprocess.run([HIPCC, "-x", "hip", *HIP_FLAGS, "-I" + work, "-c", s, "-o", o], check=True)
        objs.append(o)
    out = os.path.join(REPO, "tools", "lab", f"libpk_comm_{name}.so")
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *objs, "-o", out], check=True)
    shutil.rmtree(work, ignore_errors=True)
    return out


def build(name: str) -> str:
    if name in COMM_VARIANTS:
        return build_comm(name)
    src = os.path.join(REPO, "csrc", "kernels")
    work = tempfile.mkdtemp(prefix=f"pkvar_{name}_")
    kdir = os.path.join(work, "kernels")
    shutil.copytree(src, kdir)
    shutil.copytree(os.path.join(REPO, "csrc", "comm"), os.path.join(work, "comm"))  # comm/signals.h
    for fname, old, new in VARIANTS[name]:
        p = os.path.join(kdir, fname)
        text = open(p).read()
        if old not in text:
            raise SystemExit(f"variant {name}: pattern not found in {fname}: {old!r}")
        open(p, "w").write(text.replace(old, new))
    objs = []

    def one(s):
        o = os.path.join(work, os.path.basename(s) + ".o")
        subprocess.run([HIPCC, "-x", "hip", *HIP_FLAGS, "-I" + work, "-c", s, "-o", o], check=True)
        return o

    with cf.ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(one, sorted(glob.glob(os.path.join(kdir, "*.hip")))))
    out = os.path.join(REPO, "tools", "lab", f"libpk_kernels_{name}.so")
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", *objs, "-o", out], check=True)
    shutil.rmtree(work, ignore_errors=True)
    return out


if __name__ == "__main__":
    for n in sys.argv[1:] or list(VARIANTS) + list(COMM_VARIANTS):
        print(build(n), flush=True)
