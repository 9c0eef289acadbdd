"""Where the batched C3 launch spends its wall time (diagnostic build).

    make -C shockwave-replication_amd/csrc stamps && python tools/placement.py [batch]

The stamps build records per instance the 100 MHz wall clock at entry and
exit, HW_ID and XCC_ID.  This prints the launch span, how busy each CU was,
the gaps between consecutive workgroups on a CU, whether workgroups overlap
on a CU (co-residency), the per-XCD finish times, and the ratio of the
s_memtime phase cycles to wall time (the shader clock the stamps count)."""
import ctypes as C
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "shockwave-replication_amd"))
import sw_native as sn  # noqa: E402
import sw_synth as ss  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    lib = sn.load(os.path.join(ROOT, "shockwave-replication_amd", "lib", "libshockwave_amd_stamps.so"))
    lib.sw_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    s = sn.Solver(device=0, lib=lib)
    s.upload([ss.c3_problem(i) for i in range(B)])
    s.run()  # warm
    s.run()
    s.download()
    st = np.zeros(B * 16, dtype=np.uint64)
    lib.sw_debug_stamps(s.h, st.ctypes.data_as(C.POINTER(C.c_uint64)))
    s.close()
    st = st.reshape(B, 16)
    hw = st[:, 6] & 0xFFFFFFFF
    xcc = (st[:, 6] >> 32) & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    t0, t1 = st[:, 7].astype(np.int64), st[:, 14].astype(np.int64)
    cyc = st[:, :6].astype(np.float64).sum(axis=1) / 2.0  # two runs accumulated
    # the stamps accumulate over both runs; wall clock is the last run's
    span = (t1.max() - t0.min()) / 100.0  # µs
    dur = (t1 - t0) / 100.0
    print(f"batch {B}: launch span {span:.1f} us; mean instance wall {dur.mean():.1f} us "
          f"(min {dur.min():.1f}, max {dur.max():.1f})")
    print(f"stamped cycles / wall us (phase clock, MHz): {np.mean(cyc / np.maximum(dur, 1e-9)):.0f}")
    cus = defaultdict(list)
    for i in range(B):
        cus[(int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i]))].append((int(t0[i]), int(t1[i])))
    busy, gaps, overl, counts = [], [], 0, []
    for k, v in cus.items():
        v.sort()
        counts.append(len(v))
        busy.append(sum(b - a for a, b in v) / 100.0)
        for (a0, b0), (a1, b1) in zip(v, v[1:]):
            if a1 < b0:
                overl += 1
            else:
                gaps.append((a1 - b0) / 100.0)
    print(f"CUs used {len(cus)}; WGs per CU min {min(counts)} max {max(counts)}; "
          f"overlapping consecutive WGs on a CU: {overl}")
    print(f"busy per CU: mean {np.mean(busy):.1f} us = {100 * np.mean(busy) / span:.1f}% of the span")
    if gaps:
        print(f"gap between WGs on a CU: mean {np.mean(gaps):.2f} us, max {np.max(gaps):.2f} us")
    fin = defaultdict(int)
    beg = defaultdict(lambda: 1 << 62)
    for i in range(B):
        fin[int(xcc[i])] = max(fin[int(xcc[i])], int(t1[i]))
        beg[int(xcc[i])] = min(beg[int(xcc[i])], int(t0[i]))
    base = t0.min()
    print("per XCD first start / last finish (us from launch start):",
          {k: (round((beg[k] - base) / 100.0, 1), round((fin[k] - base) / 100.0, 1)) for k in sorted(fin)})


if __name__ == "__main__":
    main()
