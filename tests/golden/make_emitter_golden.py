"""Extract the reference's QuorumIndexer golden vector into JSON.

Run here (needs /root/reference, read as text only):
    python tests/golden/make_emitter_golden.py

Writes ``tests/golden/emitter_golden.json`` from
``emitter/ancestor/quorum_indexer_test.go:22-76`` (TestCasualityStrategy):

* ``scheme``   -- the ASCII DAG (input; event names are <name>.<stage>);
* ``weights``  -- the validator weights in node (column) order, from the
                  ``pos.ArrayToValidators(nodes, ...)`` call (:107);
* ``cap``      -- the cap of the test's capFn (:117-122);
* ``expected`` -- per stage, per node name, the chosen parents as the test
                  prints them (``parentsToString``, :201-214: self-parent
                  first, the rest sorted by name).

The fixture is data (inputs and expected outputs); no reference source text is
kept under tests/.
"""

import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    src = open(os.path.join(REF, "emitter/ancestor/quorum_indexer_test.go"), encoding="utf-8").read()
    body = src[src.index("func TestCasualityStrategy"):src.index("// testSpecialNamedParents")]
    scheme = re.search(r"`([^`]*)`", body).group(1)
    expected = {}
    for stage, block in re.findall(r"(\d+):\s*\{([^}]*)\}", body):
        expected[stage] = dict(re.findall(r'"(node\w)":\s*"(\[[^"]*\])"', block))
    w = re.search(r"ArrayToValidators\(nodes, \[\]pos\.Weight\{([^}]*)\}\)", src).group(1)
    weights = [int(x) for x in w.split(",")]
    cap = int(re.search(r"if diff > (\d+) \{", src).group(1))
    out = {"source": "emitter/ancestor/quorum_indexer_test.go:22-76 (TestCasualityStrategy)",
           "scheme": scheme, "weights": weights, "cap": cap, "expected": expected}
    with open(os.path.join(HERE, "emitter_golden.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print("stages %d, weights %s, cap %d" % (len(expected), weights, cap))


if __name__ == "__main__":
    main()
