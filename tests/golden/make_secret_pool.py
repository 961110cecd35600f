#!/usr/bin/env python3
"""Dev-time: sample planted-secret strings for the synthetic corpora.

For each builtin rule (trivy_amd/secret/builtin_rules.json) draw strings from
the rule regex's language with tests/regex_sampler.py (ASCII-biased), keeping
only samples the oracle confirms as matches.  Output: tests/golden/secret_pool.json
(data: {rule_id: [sample, ...]}), used by bench.py's corpus generator.
"""
import json
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle.goregexp import GoRegexp  # noqa: E402
from tests.regex_sampler import sample_regex  # noqa: E402


def main(per_rule=24):
    rules = json.loads((HERE.parent.parent / "trivy_amd/secret/builtin_rules.json").read_text())["rules"]
    rng = random.Random(0x5EC2E7)
    pool = {}
    for r in rules:
        rx = GoRegexp(r["regex"])
        out = []
        tries = 0
        while len(out) < per_rule and tries < per_rule * 50:
            tries += 1
            s = sample_regex(r["regex"], rng, maxrep=3)
            if any(b >= 0x80 for b in s) or b"\n" in s[:-1]:
                continue
            cand = b" " + s + b" \n"
            if rx.find_all_index(cand):
                out.append(s.decode("ascii"))
        pool[r["id"]] = out
    (HERE / "secret_pool.json").write_text(json.dumps(pool, indent=0) + "\n")
    print("rules %d, samples %d" % (len(pool), sum(len(v) for v in pool.values())))


if __name__ == "__main__":
    main()
