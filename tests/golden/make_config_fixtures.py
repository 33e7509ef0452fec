"""Collects the reference's shadow.yaml corpus as test DATA into reference_configs.json.

Inputs (all read as text from /root/reference, never executed):
* every *.yaml under src/test/ and examples/ (the configurations the reference's own
  integration tests run, src/test/CMakeLists.txt add_shadow_tests), with the CLI arguments
  that harness appends (src/test/CMakeLists.txt:62-110) and its EXPECT_ERROR flags;
* the GML graph files those configs reference by relative path (src/test/compressed-graph);
* MyTest/shadow.yaml with the reference's own output for it,
  MyTest/shadow.data/processed-config.yaml (written by core/manager.rs:253) — the golden
  vector of the configuration merge.

Run once in the build container:  python tests/golden/make_config_fixtures.py
"""
import json
import pathlib
import re

REF = pathlib.Path("/root/reference")
OUT = pathlib.Path(__file__).resolve().parent / "reference_configs.json"

# add_shadow_tests appends these unless the test's ARGS already name them
HARNESS_ARGS = ["--use-cpu-pinning", "false", "--strace-logging-mode", "standard",
                "--parallelism", "1", "--report-errors-to-stderr", "false"]


_KEYWORDS = {"BASENAME", "LOGLEVEL", "SHADOW_CONFIG", "POST_CMD", "EXPECT_ERROR", "ARGS",
             "CONFIGURATIONS", "PROPERTIES"}


def shadow_tests():
    """Every add_shadow_tests(...) call whose config is a literal file: the argv the harness
    builds (src/test/CMakeLists.txt:62-131) and whether it expects Shadow to fail."""
    out = []
    for cm in sorted(REF.glob("src/test/**/CMakeLists.txt")):
        text = re.sub(r"#[^\n]*", "", cm.read_text())
        for m in re.finditer(r"add_shadow_tests\(([^)]*)\)", text):
            toks = re.findall(r'"[^"]*"|\S+', m.group(1))
            kv, key = {}, None
            for t in toks:
                if t in _KEYWORDS:
                    key = t
                    kv.setdefault(key, [])
                elif key:
                    kv[key].append(t.strip('"'))
            base = kv["BASENAME"][0]
            cfg = kv.get("SHADOW_CONFIG", ["${CMAKE_CURRENT_SOURCE_DIR}/" + base + ".yaml"])[0]
            if not cfg.startswith("${CMAKE_CURRENT_SOURCE_DIR}/") or "$" in cfg[28:]:
                continue  # generated per configuration (e.g. "${CONFIG}")
            rel = (cm.parent / cfg[len("${CMAKE_CURRENT_SOURCE_DIR}/"):]).relative_to(REF).as_posix()
            args = list(kv.get("ARGS", []))
            joined = " ".join(args)
            for flag, val in zip(HARNESS_ARGS[::2], HARNESS_ARGS[1::2]):
                if flag not in joined:
                    args += [flag, val]
            level = (kv.get("LOGLEVEL") or ["info"])[0]
            out.append({"name": base + "-shadow", "config": rel,
                        "argv": [f"--data-directory={base}-shadow.data", f"--log-level={level}",
                                 *args, rel],
                        "expect_error": (kv.get("EXPECT_ERROR") or ["FALSE"])[0] == "TRUE"})
    return out


def main():
    tests = shadow_tests()
    errs = {t["config"] for t in tests if t["expect_error"]}
    corpus = {}
    for p in sorted(list(REF.glob("src/test/**/*.yaml")) + list(REF.glob("examples/**/*.yaml"))):
        rel = p.relative_to(REF).as_posix()
        corpus[rel] = {
            "text": p.read_text(encoding="utf-8"),
            "expect_error": rel in errs,
        }
    graphs = {}
    for rel, c in corpus.items():
        for m in re.finditer(r"path:\s*(\S+\.gml)", c["text"]):
            g = (REF / rel).parent / m.group(1)
            if g.exists():
                graphs[(pathlib.PurePosixPath(rel).parent / m.group(1)).as_posix()] = g.read_text()
    for g in REF.glob("src/test/**/*.gml"):
        graphs[g.relative_to(REF).as_posix()] = g.read_text()
    doc = {
        "_about": "Data collected from the reference by tests/golden/make_config_fixtures.py",
        "harness_args": HARNESS_ARGS,
        "tests": tests,
        "corpus": corpus,
        "graphs": graphs,
        "mytest": {
            "config": (REF / "MyTest/shadow.yaml").read_text(encoding="utf-8"),
            "processed": (REF / "MyTest/shadow.data/processed-config.yaml").read_text(encoding="utf-8"),
        },
    }
    OUT.write_text(json.dumps(doc, indent=1, ensure_ascii=False) + "\n", encoding="utf-8")
    print(f"{len(tests)} harness tests, {len(corpus)} configs ({sum(c['expect_error'] for c in corpus.values())} expect errors), "
          f"{len(graphs)} graphs -> {OUT}")


if __name__ == "__main__":
    main()
