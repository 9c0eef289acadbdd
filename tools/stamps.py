"""Per-phase cycle breakdown of the plan kernel (diagnostic build).

    make -C shockwave-replication_amd/csrc stamps && python tools/stamps.py

Phases: 0 setup (constants + key rows), 1 P1 level search, 2 P1 packing
(both orders), 3 P1 bookkeeping, 4 P2 placement, 5 emit.  s_memtime ticks
are shader-clock cycles; shares are what matter (stamps add barriers).
"""
import ctypes as C
import os
import sys

import numpy as np

SLOTS = 64  # SW_STAMP_SLOTS (csrc/sw_device.h)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def main():
    path = os.environ.get("SW_STAMPS_LIB") or os.path.join(ROOT, "shockwave-replication_amd", "lib",
                                                          "libshockwave_amd_stamps.so")
    print("library:", os.path.relpath(path, ROOT))
    lib = sn.load(path)
    lib.sw_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    cases = {
        "c3_900x30_k1e5": [ss.c3_problem(i) for i in range(int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 64)],
        # scale_64gpus.json: k = 10, λ = 5; scale_128gpus.json: k = 1e-3, λ = 15
        "g64_900x20_k10": [ss.synth_problem(i, 900, 64, 20, 120.0, 10.0, 5.0) for i in range(16)],
        "g128_900x20_k1e-3": [ss.synth_problem(i, 900, 128, 20, 120.0, 1e-3, 15.0) for i in range(16)],
    }
    if "--c5" in sys.argv:  # the C5 sweep's 512 instances (bench.c5_leg's problems)
        sys.path.insert(0, ROOT)
        import bench
        cases = {"c5_sweep": ss.sweep_problems(bench.C5_INSTANCES, 900, seed0=bench.C5_SEED0, T_override=30)}
    if "--c4" in sys.argv:  # the C4 instance alone (workspace path; its exchange at 10k jobs)
        cases = {"c4_10000x30": [ss.synth_problem(77, 10000, 2848, 30, 120.0, 1e5, 5.0)]}
    names = ["setup", "p1_level_search", "p1_pack", "p1_misc", "p2_pack", "emit"]
    for name, batch in cases.items():
        s = sn.Solver(device=0, lib=lib)
        s.upload(batch)
        s.run()
        res = s.download()
        st = np.zeros(len(batch) * SLOTS, dtype=np.uint64)
        lib.sw_debug_stamps(s.h, st.ctypes.data_as(C.POINTER(C.c_uint64)))
        st = st.reshape(len(batch), SLOTS).astype(np.float64)
        st_all = st
        pk = st[:, 8:14]
        ls = st[:, 16:23]
        srt = st[:, 15]
        scans, misses, rounds = st[:, 26].mean(), st[:, 27].mean(), st[:, 25].mean()
        st = st[:, :6]
        tot = st.sum(axis=1).mean()
        print(f"{name}: mean cycles/instance {tot:.0f}; passes {np.mean([r['iters'] for r in res]):.1f}; "
              f"status {sorted(set(r['status'] for r in res))}")
        for i, n in enumerate(names):
            print(f"   {n:16s} {st[:, i].mean():12.0f}  {100 * st[:, i].mean() / tot:5.1f}%")
        pnames = ["setup", "hist+need", "tiers", "fill", "tail", "apply"]
        print("   pack round loop (all packs of an instance):",
              " ".join(f"{n} {pk[:, i].mean():.0f}" for i, n in enumerate(pnames)))
        print("   wave round loop tier parts: head {:.0f} scan {:.0f} take {:.0f} | one stamp {:.0f}".format(
            *st_all[:, 28:31].mean(axis=0), st_all[:, 31].mean() / max(rounds, 1)))
        print(f"   sorts (all packs): {srt.mean():.0f}; rounds {rounds:.1f}, active tiers {scans:.1f}, "
              f"width-tail reductions {misses:.1f}")
        print("   pack sub-phases (all packs): keys+offsets {:.0f} compaction {:.0f} loop+staging {:.0f} "
              "write-back {:.0f} | post-pack evaluation {:.0f}".format(*st_all[:, 48:53].mean(axis=0)))
        lnames = ["force", "price_probes", "tie", "tail", "eval", "M_lo", "between"]
        print("   level search:", " ".join(f"{n} {ls[:, i].mean():.0f}" for i, n in enumerate(lnames)),
              f"| price probes {st_all[:, 23].mean():.1f}, M_lo passes {st_all[:, 24].mean():.1f}")
        px = st_all[:, 32:43]
        pn = ["classes", "ranks", "bitsets", "edges", "bellman_ford", "select", "apply", "bf_iters",
              "builds", "bf_relax", "bf_walks"]
        print("   P2 exchange kernel (sw_p2x_kernel):", " ".join(
            f"{n} {px[:, i].mean():.0f}" for i, n in enumerate(pn)),
            f"| total {px[:, :7].sum(axis=1).mean():.0f}")
        if "--c5" in sys.argv:  # the slowest instances: solve + exchange cycles
            tot_i = st.sum(axis=1) + px[:, :7].sum(axis=1)
            print("   slowest instances (G, k, passes, status | solve phases | exchange phases, bf_iters, builds):")
            for i in np.argsort(-tot_i)[:12]:
                a = batch[i]
                print(f"     #{i:3d} G {a.G:3d} k {a.k:g} it {res[i]['iters']:4d} st {res[i]['status']:4d} total "
                      f"{tot_i[i]:9.0f} |", " ".join(f"{v:8.0f}" for v in st[i]), "|",
                      " ".join(f"{v:8.0f}" for v in px[i, :9]))
        if "-v" in sys.argv:  # per-instance rows: status, passes, phase cycles
            for r, row, prow in list(zip(res, st, pk))[:24]:
                print("     st", r["status"], "it", r["iters"], " ".join(f"{v:9.0f}" for v in row), "|",
                      " ".join(f"{v:8.0f}" for v in prow))
        s.close()


if __name__ == "__main__":
    main()
