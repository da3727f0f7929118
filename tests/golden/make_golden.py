"""Writes the golden fixtures of tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``).  Test data only; nothing here is
imported by the product path.

Two kinds of vector:

* ``edge_cases.json`` -- the reference's own fixtures and answers, not our
  oracle's output:
    - the 9 node sets of ``known-idempotent-insert-edge-cases``
      (list_test.cljc:44-96, transcribed in tests/refgen.py);
    - their full-reweave orders and visible EDN, derived in SURVEY.md
      Appendix B by an independent transliteration of weave-node
      (shared.cljc:194-241) made before this oracle existed;
    - the EDN answers the reference's tests assert (list_test.cljc:162-173,
      map_test.cljc:17-43 and the F8a quirk);
    - the Java ``String.compareTo`` order of the exotic site ids
      (list_test.cljc:64-95), which pins the id order of ``(sort ::nodes)``.
* ``packed_vectors.npz`` -- seeded packed-key batches (reference-style random
  histories, stress histories incl. tx chains, config-2-shaped documents)
  with the weave order, visibility, max lamport-ts and yarn order of the
  C oracle's literal fold (oracle/weave_oracle.c, checked against the literal
  Python restatement by tests/test_oracle.py).  They let the GPU tests check
  the HIP path without running the oracle, and pin the oracle against drift.
"""
from __future__ import annotations

import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from cause_amd import gen, pack  # noqa: E402
from oracle import causal_ref as R  # noqa: E402
from tests import refgen as G  # noqa: E402

# (ts, first 2 chars of site, value) after the root, and
# the visible EDN.  "hide" is :causal/hide.
APPENDIX_B = [
    ([(1, "xT", "hide"), (4, "9F", "d"), (3, "9F", "r"), (4, "Nw", " "), (2, "9F", "d")],
     ["d", "r", " ", "d"]),
    ([(2, "xT", "b"), (1, "xT", " "), (2, "Nw", "q"), (2, "9F", " ")], ["b", " ", "q", " "]),
    ([(1, "Pz", "o"), (2, "Pz", "hide"), (3, "9F", "u"), (2, "Nw", " ")], ["u", " "]),
    ([(1, "A~", "hide"), (1, "W7", "j"), (1, "Vd", "w")], ["j", "w"]),
    ([(1, "W7", "u"), (2, "7h", "hide"), (2, "W7", " "), (1, "Vd", "m")], [" ", "m"]),
    ([(1, "Ft", "hide"), (1, "A~", "hide")], []),
    ([(1, "Vd", "hide"), (3, "A~", "i"), (2, "A~", "j"), (1, "W7", "s")], ["i", "j", "s"]),
    ([(1, " f", "hide"), (2, " z", " "), (2, " f", "l"), (2, " a", "v")], [" ", "l", "v"]),
    ([(2, " f", "hide"), (1, " f", "hide"), (3, " a", "c"), (2, " z", "r")], ["c", "r"]),
]

# list_test.cljc:64-95 site ids in Java String.compareTo order
SITE_ORDER = [" a ", " f ", " z ", "0", "7hLbMKLvcll_4", "9FyYzf9pum6E4", "A~iIXinAXkGX7"]

# Answers the reference's tests assert (EDN as JSON: keywords as ":name").
KNOWN_ANSWERS = {
    "list_hide_show": {  # list_test.cljc:162-173
        "ops": ["conj a", "conj b", "conj c", "hide a", "show a", "hide a", "show a"],
        "edn_after_each": [["a", "b", "c"], ["b", "c"], ["a", "b", "c"], ["b", "c"],
                           ["a", "b", "c"]]},
    "map_hide_show": {  # map_test.cljc:17-31
        "edn_after_each": [{":foo": "bar", ":fizz": "buzz"}, {":fizz": "buzz"},
                           {":foo": "bar", ":fizz": "buzz"}, {":fizz": "buzz"},
                           {":foo": "bar", ":fizz": "buzz"}, {":foo": "boo", ":fizz": "buzz"}]},
    "map_hide_show_by_id": {  # map_test.cljc:33-43
        "edn_after_each": [{":foo": "bar"}, {":foo": "boo"}, {":foo": "bar"}, {":foo": "boo"}]},
    "map_quirk_f8a": {"edn": {}},  # assoc :a 1, dissoc :a, assoc :a 2
}


def _val(v):
    if isinstance(v, R.Keyword):
        return {"kw": (v.ns + "/" if v.ns else "") + v.name}
    return v


def _id(i):
    return None if i is None else [i[0], i[1], i[2]]


def edge_cases():
    cases = []
    for nodes, (weave, edn) in zip(G.EDGE_CASES, APPENDIX_B):
        cases.append({
            "nodes": [[_id(n[0]), _id(n[1]), _val(n[2])] for n in nodes],
            "weave_after_root": [[ts, s, "hide" if v == "hide" else v] for ts, s, v in weave],
            "edn": edn,
        })
    return {"source": "list_test.cljc:44-96 nodes; SURVEY.md Appendix B orders",
            "cases": cases, "site_order": SITE_ORDER, "known_answers": KNOWN_ANSWERS}


def _batch(docs_nodes):
    """Pack Clojure-shaped documents (root included) into one batch."""
    return pack.pack_lists(docs_nodes)


def packed_vectors():
    rng = random.Random(20261016)
    groups = {}
    # reference-style random histories (list_test.cljc:9-32 generator shape)
    docs = []
    for steps in (1, 5, 9, 20, 60, 200):
        for _ in range(4):
            nodes, _ = G.random_history(rng, steps)
            d = [R.ROOT_NODE] + nodes
            rng.shuffle(d)
            docs.append(d)
    b = _batch(docs)
    groups["refhist"] = (b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    # stress histories (hide-of-hide chains, dirty conj causes, tx chains)
    docs = []
    for steps, tx in ((30, 0.0), (120, 0.0), (400, 0.0), (300, 0.3)):
        for _ in range(3):
            d = G.stress_history(rng, steps, tx_chain=tx)  # root included
            rng.shuffle(d)
            docs.append(d)
    b = _batch(docs)
    groups["stress"] = (b.offsets, b.id_key, b.cause_key, b.kind, b.layout)
    # config-2-shaped documents (generator, 3 docs x 2,000 nodes)
    import dataclasses
    spec = dataclasses.replace(gen.CONFIG2, nodes_per_doc=2000, seed=0x601D)
    off, i, c, k = gen.generate(spec, 0, 3)
    groups["config2"] = (off, i, c, k, spec.layout())
    out = {}
    for name, (off, i, c, k, lay) in groups.items():
        perm, vis, st = oracle.batch_lists(off, i, c, k, method=oracle.METHOD_LITERAL)
        assert not st.any(), name
        D = len(off) - 1
        max_ts = np.array([(int(i[off[d]:off[d + 1]].max()) >> lay.ts_shift) if off[d + 1] > off[d]
                           else 0 for d in range(D)], np.uint64)
        yarn = np.concatenate([
            oracle.list_yarns(i[off[d]:off[d + 1]], lay.site_shift, (1 << lay.site_bits) - 1)
            for d in range(D)]).astype(np.uint32)
        out[f"{name}_offsets"] = np.asarray(off, np.uint64)
        out[f"{name}_id_key"] = np.asarray(i, np.uint64)
        out[f"{name}_cause_key"] = np.asarray(c, np.uint64)
        out[f"{name}_kind"] = np.asarray(k, np.uint8)
        out[f"{name}_layout"] = np.array([lay.ts_bits, lay.site_bits, lay.tx_bits], np.uint32)
        out[f"{name}_weave_perm"] = perm.astype(np.uint32)
        out[f"{name}_visible"] = vis.astype(np.uint8)
        out[f"{name}_max_ts"] = max_ts
        out[f"{name}_yarn_perm"] = yarn
    return out


def main():
    with open(os.path.join(HERE, "edge_cases.json"), "w") as f:
        json.dump(edge_cases(), f, indent=1, ensure_ascii=False)
        f.write("\n")
    np.savez_compressed(os.path.join(HERE, "packed_vectors.npz"), **packed_vectors())
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
