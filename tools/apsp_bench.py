"""APSP build times on the bench graphs (Tor-like complete graph, config C; random sparse
graph, config B/D) at V = 1000 and 2000, both latency forms (u32 squaring, u64
Floyd-Warshall via SGN_APSP_FW=1 in a child process). The first build of a process includes
code-object loading; later ones are the steady-state build time. Prints JSON lines."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "shadow-gen_amd"))
import numpy as np  # noqa: E402

import sgn  # noqa: E402


def run(kind, V):
    g = sgn.tor_graph(V, seed=42) if kind == "tor" else sgn.random_graph(V, seed=42)
    used = np.arange(V, dtype=np.uint32)
    ctx = sgn.Context()
    ts = []
    for i in range(4):
        ctx.routes_build(g, used)
        ts.append(ctx.routes_timing())
    t = ts[-1]
    return {"graph": kind, "V": V, "arcs": int(t["n_tight_edges"]), "first_build_ms": round(ts[0]["total_ms"], 3),
            **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in t.items()},
            "form": "per-source relaxation (u64)" if t["latency_bf"] else
                    ("u64 Floyd-Warshall" if t["latency_u64"] else "u32 min-plus squaring"),
            "loss_form": (f"dense {t['loss_multi']}-source sweep + fold" + (" (fused with the first pass)" if t.get("loss_fused") else "")
                          if t.get("loss_dense") else
                          f"{t['loss_multi']}-source sweep + fold") if t["loss_multi"] else "one-source pass"}


if __name__ == "__main__":
    if len(sys.argv) > 2:
        print(json.dumps(run(sys.argv[1], int(sys.argv[2]))), flush=True)
        sys.exit(0)
    for mode in ("default", "sq", "loss1", "fw"):
        for kind in ("tor", "random"):
            for V in (1000, 2000):
                env = dict(os.environ)
                env.pop("SGN_APSP_FW", None)
                env.pop("SGN_APSP_LOSS1", None)
                env.pop("SGN_APSP_SQ", None)
                if mode == "sq":
                    env["SGN_APSP_SQ"] = "1"
                elif mode == "fw":
                    env["SGN_APSP_FW"] = "1"
                elif mode == "loss1":
                    env["SGN_APSP_LOSS1"] = "1"
                r = subprocess.run([sys.executable, __file__, kind, str(V)], env=env, capture_output=True, text=True)
                sys.stdout.write(r.stdout)
                if r.returncode:
                    sys.stderr.write(r.stderr)
                    sys.exit(r.returncode)
