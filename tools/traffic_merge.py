"""Files keyed PMC traffic entries (tools/pmc_traffic.py output, argv[1:]) into
profiles/round_kernel_traffic.json ({"entries": [...]}, one per bench invocation)."""
import json
import pathlib
import sys

out = pathlib.Path(__file__).resolve().parent.parent / "profiles" / "round_kernel_traffic.json"
cur = json.loads(out.read_text()) if out.exists() else {}
entries = cur.get("entries", [])
for f in sys.argv[1:]:
    e = json.loads(pathlib.Path(f).read_text())
    key = lambda x: (json.dumps(x["workload"], sort_keys=True), x["kernel"])  # noqa: E731
    # (an invocation's entry replaces the older one, whatever build that was measured on)
    entries = [x for x in entries if key(x) != key(e)] + [e]
out.write_text(json.dumps({"entries": entries}, indent=1) + "\n")
print(f"{out}: {len(entries)} entries")
