"""Generate reference-pinned quorum and vote-tally fixtures by running the
reference's own plenum/server/quorums.py (Quorums, with getMaxFailures taken
from plenum/common/util.py:217-228 as written) and plenum/server/models.py
(TrackedMsgs / Prepares / Commits) in THIS container:

    /opt/conda/bin/python3.9 tests/golden/gen_ref_quorums.py

Outputs (pure data, committed):
  quorums_kat.json   Quorums(n).__dict__ values for n = 1..63
  tally_kat.json     vote streams -> the distinct-voter sets Prepares/Commits
                     hold and their hasQuorum() verdicts at Quorums(n).prepare /
                     .commit, per (viewNo, ppSeqNo) key

What the replica does before a vote reaches Prepares.addVote is restated here
(Replica.validatePrepare, plenum/server/replica.py:1289-1291): a PREPARE from
the primary of its view raises SuspiciousNode(PR_FRM_PRIMARY) and is never
added.  Votes whose signature / precondition failed (valid = 0) are never
added either (the message is discarded before processPrepare/processCommit).
Duplicates from one voter are added once (set semantics, models.py:21-25; the
replica also flags them, replica.py:1295-1297).
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_standins as R  # noqa: E402

R.install()
from plenum.server.quorums import Quorums  # noqa: E402
from plenum.server.models import Prepares, Commits  # noqa: E402
from plenum.common.messages.node_messages import Prepare, Commit  # noqa: E402

PREPARE, COMMIT = 0, 1


def quorums_kat():
    out = []
    for n in range(1, 64):
        q = Quorums(n)
        row = {"n": n, "f": q.f}
        for name, v in q.__dict__.items():
            if name != "f":
                row[name] = v.value
        out.append(row)
    return out


def run_votes(n, keys, primary, votes):
    """Feed votes through the reference's Prepares / Commits."""
    q = Quorums(n)
    prepares, commits = Prepares(), Commits()
    names = ["Node%d" % (v + 1) for v in range(n)]
    for k, voter, phase, valid in votes:
        if not valid:
            continue
        view, seq = keys[k]
        if phase == PREPARE:
            if voter == primary[k]:  # replica.py:1289-1291: PREPARE from the primary
                continue
            prepares.addVote(Prepare(0, view, seq, 0, "d", "s", "t"), names[voter])
        else:
            commits.addVote(Commit(0, view, seq), names[voter])
    counts, prepared, committed = [], [], []
    for view, seq in keys:
        p, c = Prepare(0, view, seq, 0, "d", "s", "t"), Commit(0, view, seq)
        counts.append([len(prepares[(view, seq)].voters) if prepares.hasPrepare(p) else 0,
                       len(commits[(view, seq)].voters) if commits.hasCommit(c) else 0])
        prepared.append(bool(prepares.hasQuorum(p, q.prepare.value)))
        committed.append(bool(commits.hasQuorum(c, q.commit.value)))
    return {"counts": counts, "prepared": prepared, "committed": committed,
            "prepare_quorum": q.prepare.value, "commit_quorum": q.commit.value}


def scenario(name, n, n_keys, rng, p_valid=0.95, p_dup=0.1, density=0.8):
    keys = [[k // 7, k + 1] for k in range(n_keys)]
    primary = [view % n for view, _ in keys]
    votes = []
    for k in range(n_keys):
        for phase in (PREPARE, COMMIT):
            for v in range(n):
                if rng.random() < density:
                    votes.append([k, v, phase, int(rng.random() < p_valid)])
                    if rng.random() < p_dup:
                        votes.append([k, v, phase, int(rng.random() < p_valid)])
    rng.shuffle(votes)
    return {"name": name, "n": n, "keys": keys, "primary": primary, "votes": votes,
            "expect": run_votes(n, keys, primary, votes)}


def edge_scenarios():
    out = []
    # n = 4: prepare quorum 2.  Key 0 has PREPAREs from the primary (0) and
    # node 1 only -- it would reach 2 if the primary's PREPARE counted.
    n, keys, primary = 4, [[0, 1], [0, 2], [1, 3]], [0, 0, 1]
    votes = [[0, 0, PREPARE, 1], [0, 1, PREPARE, 1],
             [1, 1, PREPARE, 1], [1, 2, PREPARE, 1], [1, 1, PREPARE, 1],
             [2, 0, PREPARE, 1], [2, 1, PREPARE, 1], [2, 2, PREPARE, 0],
             [0, 0, COMMIT, 1], [0, 1, COMMIT, 1], [0, 2, COMMIT, 1],
             [1, 3, COMMIT, 1], [1, 3, COMMIT, 1], [1, 2, COMMIT, 1]]
    out.append({"name": "primary-prepare-would-reach-quorum", "n": n, "keys": keys, "primary": primary,
                "votes": votes, "expect": run_votes(n, keys, primary, votes)})
    # n = 25 (configs[4]): prepare 16, commit 17; key 0 has exactly 15 non-primary
    # PREPAREs plus the primary's, key 1 has 16 non-primary ones
    n, keys, primary = 25, [[3, 10], [3, 11]], [3, 3]
    votes = []
    for v in range(25):
        if v == 3 or len([x for x in votes if x[0] == 0]) < 15:
            votes.append([0, v, PREPARE, 1])
    votes += [[1, v, PREPARE, 1] for v in range(25) if v != 3][:16]
    votes += [[0, v, COMMIT, 1] for v in range(16)] + [[1, v, COMMIT, 1] for v in range(17)]
    votes += [[1, 0, COMMIT, 1]] * 3
    out.append({"name": "n25-thresholds", "n": n, "keys": keys, "primary": primary, "votes": votes,
                "expect": run_votes(n, keys, primary, votes)})
    # no votes at all / one voter
    out.append({"name": "empty", "n": 7, "keys": [[0, 1]], "primary": [0], "votes": [],
                "expect": run_votes(7, [[0, 1]], [0], [])})
    return out


def tally_kat():
    rng = random.Random(2024)
    cases = edge_scenarios()
    for n in (4, 7, 10, 25):
        cases.append(scenario("random-n%d" % n, n, 40, rng))
    cases.append(scenario("random-n25-sparse", 25, 60, rng, p_valid=0.9, p_dup=0.3, density=0.65))
    return cases


def main():
    with open(os.path.join(HERE, "quorums_kat.json"), "w") as f:
        json.dump(quorums_kat(), f, indent=0)
    with open(os.path.join(HERE, "tally_kat.json"), "w") as f:
        json.dump(tally_kat(), f, separators=(",", ":"))
    print("ok")


if __name__ == "__main__":
    main()
