"""Extract the reference's golden vectors for the vector-clock / FC path into JSON.

Run here (needs /root/reference, read as text only):
    python tests/golden/make_golden.py

Writes ``tests/golden/fc_golden.json`` with, for each case, the ASCII DAG
(input) and the expected ForklessCause relation (output) exactly as the
reference tests state them:

* ``vecfc/forkless_cause_test.go:82-123`` (TestForklessCausedClassic, 3 DAGs).
  Expected FC(who, whom) <=> bylevel(whom) > 0 and bylevel(whom) <= level(who),
  decoded from the event names per ``:128-193``; we expand the rule into the
  explicit pair list here so the fixture is plain data.
* ``vecfc/forkless_cause_test.go:199-441`` (TestForklessCausedRandom): the
  80-event, 4-validator DAG and its full expected FC relation table.
* ``vecfc/forkless_cause_test.go:29-40`` (BenchmarkIndex_ForklessCause's
  15-validator DAG; no expected output, used as a parity input only).
* ``abft/event_processing_root_test.go`` (TestLachesisClassicRoots /
  TestLachesisRandomRoots): DAGs whose event names encode frame and root-ness
  (``:251-301``), kept for the abft restatement row.
* ``abft/election/election_test.go:35-170`` (TestProcessRoot, 5 cases) ->
  ``abft_golden.json``: ASCII DAG, validator weights by node name, and the
  expected decided frame, Atropos name and decisive roots.  The observe
  relation of that test is "direct parent edge" (``:213-232``), minus the
  self-parent of events whose name starts with ``+``.

The fixture is data (inputs and expected outputs); no reference source text is
kept under tests/.
"""

import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def backtick_blocks(src):
    return re.findall(r"`([^`]*)`", src)


def decode_level(name):
    # forkless_cause_test.go:172-193
    s = name.split("_")[1].split("(")
    level = int(s[0])
    bylevel = int(s[1].rstrip(")")) if len(s) > 1 else 0
    return level, bylevel


def names_in(scheme):
    out = []
    for line in scheme.strip().split("\n"):
        for sym in re.split("[ ─═]+", line.strip()):
            if not sym or sym.startswith("//"):
                if sym.startswith("//"):
                    break
                continue
            if re.match(r"^[A-Za-z]", sym):
                out.append(sym)
    return out


def main():
    fc_src = open(os.path.join(REF, "vecfc/forkless_cause_test.go"), encoding="utf-8").read()
    blocks = backtick_blocks(fc_src)
    # order in file: bench scheme, classic x3, random scheme
    bench_scheme, c3, c4, c5, rnd = blocks[0], blocks[1], blocks[2], blocks[3], blocks[4]

    cases = []
    for label, sch in (("classic_step3", c3), ("classic_step4", c4), ("classic_step5", c5)):
        names = names_in(sch)
        rel = {}
        for who in names:
            lvl, _ = decode_level(who)
            rel[who] = sorted(w for w in names
                              if decode_level(w)[1] > 0 and decode_level(w)[1] <= lvl)
        cases.append({"name": label, "source": "vecfc/forkless_cause_test.go:82-123",
                      "scheme": sch, "weights": "equal1", "fc": rel})

    # relations table of TestForklessCausedRandom (:360-441)
    m = re.search(r"relations := map\[string\]map\[string\]struct\{\}\{(.*?)\n\t\}\n", fc_src, re.S)
    rel = {}
    for line in m.group(1).strip().split("\n"):
        mm = re.match(r'\s*"(\w+)": map\[string\]struct\{\}\{(.*)\},\s*$', line)
        who = mm.group(1)
        rel[who] = sorted(re.findall(r'"(\w+)"', mm.group(2)))
    cases.append({"name": "random_80", "source": "vecfc/forkless_cause_test.go:195-483",
                  "scheme": rnd, "weights": "equal1", "fc": rel})
    cases.append({"name": "bench_15", "source": "vecfc/forkless_cause_test.go:29-40",
                  "scheme": bench_scheme, "weights": "equal1", "fc": None})

    roots_src = open(os.path.join(REF, "abft/event_processing_root_test.go"), encoding="utf-8").read()
    rb = backtick_blocks(roots_src)
    roots = [{"name": "classic_roots", "source": "abft/event_processing_root_test.go:15-74",
              "scheme": rb[0]},
             {"name": "random_roots", "source": "abft/event_processing_root_test.go:76-239",
              "scheme": rb[1]}]

    out = {"generated_by": "tests/golden/make_golden.py", "fc_cases": cases, "roots_cases": roots}
    with open(os.path.join(HERE, "fc_golden.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print("wrote", len(cases), "fc cases,", len(roots), "root cases")

    el_src = open(os.path.join(REF, "abft/election/election_test.go"), encoding="utf-8").read()
    el_cases = []
    for m in re.finditer(r't\.Run\("([^"]+)", func\(t \*testing\.T\) \{\s*testProcessRoot\(t,(.*?)`(.*?)`\)', el_src, re.S):
        label, body, scheme = m.group(1), m.group(2), m.group(3)
        exp = None
        if "&testExpected" in body:
            fr = int(re.search(r"DecidedFrame:\s*(\d+)", body).group(1))
            at = re.search(r'DecidedAtropos:\s*"(\w+)"', body).group(1)
            dec = re.search(r"DecisiveRoots:\s*map\[string\]bool\{(.*?)\}", body).group(1)
            exp = {"frame": fr, "atropos": at, "decisive": sorted(re.findall(r'"([+\w]+)":\s*true', dec))}
        w = {}
        for nm, expr in re.findall(r'"(node\w)":\s*([^,\n]+),', body):
            expr = expr.replace("math.MaxUint32", str(0xFFFFFFFF)).replace("/", "//")
            w[nm] = int(eval(expr, {"__builtins__": {}}))
        el_cases.append({"name": label, "source": "abft/election/election_test.go:35-170",
                         "scheme": scheme, "weights": w, "expected": exp})
    out2 = {"generated_by": "tests/golden/make_golden.py", "election_cases": el_cases}
    with open(os.path.join(HERE, "abft_golden.json"), "w", encoding="utf-8") as f:
        json.dump(out2, f, ensure_ascii=False, indent=1)
    print("wrote", len(el_cases), "election cases")


if __name__ == "__main__":
    sys.exit(main())
