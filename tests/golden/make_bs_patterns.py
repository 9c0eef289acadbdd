"""Generate tests/golden/bs_patterns.json from the REFERENCE's own batch-size
pattern functions.

Run in the build container only (the reference is not on the GPU box):

    python tests/golden/make_bs_patterns.py

``scheduler/utils.py`` cannot be imported here (it imports cvxpy through the
policies package), so this script parses it with ``ast``,
takes exactly three pure functions — get_accordion_bs_pattern
(utils.py:635-688), get_accordion_in_critical_regime (:691-710) and
get_gns_bs_pattern (:713-1180) — and executes them, unmodified, over every
(model, batch size, scale factor) of the v100 throughput table and a spread
of epoch counts around every segment boundary.  Only their outputs (data)
are written; no reference source is stored.
"""
import ast
import json
import os

REF_UTILS = "/root/reference/scheduler/utils.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "bs_patterns.json")
FUNCS = ("get_accordion_bs_pattern", "get_accordion_in_critical_regime", "get_gns_bs_pattern")


def load_reference_functions():
    tree = ast.parse(open(REF_UTILS).read())
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in FUNCS]
    assert len(body) == len(FUNCS)
    ns = {}
    exec(compile(ast.Module(body=body, type_ignores=[]), REF_UTILS, "exec"), ns)
    return [ns[f] for f in FUNCS]


def rle(seq):
    """[(value, run length), …] — keeps the fixture small."""
    out = []
    for v in seq:
        if out and out[-1][0] == v:
            out[-1][1] += 1
        else:
            out.append([v, 1])
    return out


def main():
    acc_pattern, acc_critical, gns_pattern = load_reference_functions()
    cases = [
        ("ResNet-18", [16, 32, 64, 128, 256]), ("ResNet-50", [16, 32, 64, 128]),
        ("Transformer", [16, 32, 64, 128]), ("LM", [5, 10, 20, 40, 80]),
        ("Recommendation", [512, 1024, 2048, 4096, 8192]),
    ]
    epochs = sorted(set([1, 2, 3, 5, 9, 10, 11, 12, 13, 20, 21, 22, 23, 30, 31, 32, 33, 40, 41, 42,
                         43, 50, 51, 52, 60, 61, 62, 63, 70, 71, 72, 73, 80, 81, 82, 90, 91, 92, 93,
                         100, 101, 102, 103, 110, 111, 112, 113, 130, 131, 132, 133, 150, 160, 190,
                         191, 192, 193, 220, 221, 222, 223, 250, 260, 300, 500, 760, 761]))
    gns, acc, crit = [], [], []
    for model, sizes in cases:
        for bs in sizes:
            job_type = f"{model} (batch size {bs})"
            for E in epochs:
                acc.append({"job_type": job_type, "bs": bs, "E": E,
                            "out": rle(acc_pattern(job_type, bs, E))})
                for sf in (1, 2, 4, 8):
                    gns.append({"job_type": job_type, "bs": bs, "E": E, "sf": sf,
                                "out": rle(gns_pattern(job_type, bs, E, sf))})
            if model != "Transformer":
                crit.append({"model": model, "bs": bs,
                             "out": rle([bool(acc_critical(model, bs, e)) for e in range(700)])})
    json.dump({"gns": gns, "accordion": acc, "critical": crit}, open(OUT, "w"),
              separators=(",", ":"))
    print(f"wrote {OUT}: {len(gns)} gns, {len(acc)} accordion, {len(crit)} critical cases")


if __name__ == "__main__":
    main()
