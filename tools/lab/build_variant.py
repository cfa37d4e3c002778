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
    # round 6 ablations of the 4-wave prefill GEMM (timing only, wrong results;
    # profiles/r6_prefill_gemm_buffer_lds.md): no vmcnt wait before the tile barrier, no staging
    # loads in the k-loop (double-buffer form: gate_up 1,350 / 1,151 vs 1,393 us -- the loads' issue
    # cost, not their latency)
    "pb_novm": [("gemm_prefill.hip", "if constexpr (BW >= 0) wait_vm<BW>();", "")],
    "pb_noload": [("gemm_prefill.hip", "if constexpr (C == 1) stage_w(mf, lt);\n        else stage_a(mf, lt);",
                   "(void)lt;")],
    # round 6, measured and removed (profiles/r6_prefill_gemm_buffer_lds.md): sc0 / nt cache policy on
    # the staging loads ("pb_sc0_w", "pb_sc0_a": no change; "pb_nt_w": down -6 %, gate_up +4 %, O
    # +7 %), W loads moved to the even sub-step of the double buffer ("pb_split": -6 to -13 %), no XOR
    # chunk swizzle ("pb_noswz": 1,328 vs 1,330 us at gate_up)
    # round 6, measured and removed: a four-deep weight ring in the fused MLP's gate_up tiles only
    # (one workgroup per CU there, so the extra registers cost no occupancy): 8B decode step
    # 3.982-3.999 vs 3.984-3.986 ms -- the stream is not short of bytes in flight (r6_wdeep.jsonl)
    # round 6, measured and removed: the fused MLP's down tiles reading the in-launch h hand-off with
    # plain loads ("h_plain", timing only, not coherent: 3.974 vs 3.973-3.984 ms per 8B step) or plain
    # loads after one agent-scope acquire per wave ("h_acq", coherent: 4.18 ms) instead of sc1 loads
    # -- the sc1 re-reads of h cost nothing measurable (profiles/r6_hload.jsonl)
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
