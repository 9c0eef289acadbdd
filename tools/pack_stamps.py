"""Round-loop phase cycles of the sharded placement kernel (diagnostic build).

    make -C shockwave-replication_amd/csrc stamps && python tools/pack_stamps.py

Solves one C4 instance on the sharded engine at world 1 with the stamps
library and prints the cycles per phase of k_pack_rounds (thread 0's
s_memtime view; shader-clock cycles, summed over the solve's packs) and the
loop's counters: rounds, active tiers, width-tail reductions."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402

NAMES = ["setup", "hist+need", "tiers", "fill", "tail", "apply"]


def main():
    lib = sn.load(os.path.join(ROOT, "shockwave-replication_amd", "lib", "libshockwave_amd_stamps.so"))
    lib.sw_debug_pack_stamps.argtypes = [C.POINTER(C.c_uint64)]
    for N, G in ((900, 256), (10000, 2848)):
        a = ss.synth_problem(5, N, G, 30, 120.0, 1e5, 5.0)
        s = sn.Solver(device=0, lib=lib)
        s.dist_init(sn.unique_id(lib), 0, 1)
        s.dist_solve(a, 0, a.N)
        out = (C.c_uint64 * 24)()
        lib.sw_debug_pack_stamps(out)
        s.dist_solve(a, 0, a.N)
        lib.sw_debug_pack_stamps(out)
        tot = sum(out[:6])
        print(f"N={N}: round-loop cycles per solve {tot}")
        for i, n in enumerate(NAMES):
            print(f"   {n:10s} {out[i]:10d} {100.0 * out[i] / max(tot, 1):5.1f}%")
        print(f"   rounds {out[17]}  tiers {out[18]}  tail reductions {out[19]}")
        s.close()


if __name__ == "__main__":
    main()
