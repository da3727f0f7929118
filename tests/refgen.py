"""History generators shaped like the reference's own test generators.

* ``rand_node`` / ``insert_rand_nodes`` -- list_test.cljc:9-32 (random cause among
  all nodes, ts = 1 + max(cause ts, the site's yarn ts), values from
  ``simple-values`` incl. specials and the *normal* keyword ``:s/h.show``).
* ``rand_weave_of_phrases`` -- list_test.cljc:118-155.
* ``EDGE_CASES`` -- the 9 node sets of known-idempotent-insert-edge-cases,
  list_test.cljc:44-96 (data, transcribed as Python tuples).
* ``stress_history`` -- wider random histories (hide-of-hide chains, dirty
  conj-style causes, tx chains) for the F4/F5 equivalence properties.
"""
from __future__ import annotations

import random

from oracle import causal_ref as R

HIDE, H_HIDE, H_SHOW = R.HIDE, R.H_HIDE, R.H_SHOW
S_H_SHOW = R.Keyword("s", "h.show")  # a NORMAL keyword (list_test.cljc:10)

# list_test.cljc:9-10
SIMPLE_VALUES = ([HIDE, HIDE, H_HIDE, H_HIDE, S_H_SHOW, S_H_SHOW, " ", " ", " ", " ", "\n"]
                 + [chr(c) for c in range(97, 97 + 26)])

ROOT = R.ROOT_ID

# list_test.cljc:44-96
EDGE_CASES = [
    [((1, "xT_odlTBwTRNU", 0), ROOT, HIDE),
     ((2, "9FyYzf9pum6E4", 0), (1, "xT_odlTBwTRNU", 0), "d"),
     ((3, "9FyYzf9pum6E4", 0), ROOT, "r"),
     ((4, "NwudSBdQg3Ru2", 0), (3, "9FyYzf9pum6E4", 0), " "),
     ((4, "9FyYzf9pum6E4", 0), ROOT, "d")],
    [((1, "xT_odlTBwTRNU", 0), ROOT, " "),
     ((2, "xT_odlTBwTRNU", 0), ROOT, "b"),
     ((2, "NwudSBdQg3Ru2", 0), (1, "xT_odlTBwTRNU", 0), "q"),
     ((2, "9FyYzf9pum6E4", 0), (1, "xT_odlTBwTRNU", 0), " ")],
    [((1, "Pz8iuNCXvVsYN", 0), ROOT, "o"),
     ((2, "Pz8iuNCXvVsYN", 0), (1, "Pz8iuNCXvVsYN", 0), HIDE),
     ((3, "9FyYzf9pum6E4", 0), (2, "Pz8iuNCXvVsYN", 0), "u"),
     ((2, "NwudSBdQg3Ru2", 0), (1, "Pz8iuNCXvVsYN", 0), " ")],
    [((1, "W7XhooU1Hsw7E", 0), ROOT, "j"),
     ((1, "VdIJLRISw~zgo", 0), ROOT, "w"),
     ((1, "A~iIXinAXkGX7", 0), ROOT, HIDE)],
    [((1, "W7XhooU1Hsw7E", 0), ROOT, "u"),
     ((2, "W7XhooU1Hsw7E", 0), (1, "W7XhooU1Hsw7E", 0), " "),
     ((2, "7hLbMKLvcll_4", 0), (1, "W7XhooU1Hsw7E", 0), HIDE),
     ((1, "VdIJLRISw~zgo", 0), ROOT, "m")],
    [((1, "Ftbpo0oG7ZnpR", 0), ROOT, HIDE),
     ((1, "A~iIXinAXkGX7", 0), ROOT, HIDE)],
    [((1, "VdIJLRISw~zgo", 0), ROOT, HIDE),
     ((2, "A~iIXinAXkGX7", 0), (1, "VdIJLRISw~zgo", 0), "j"),
     ((3, "A~iIXinAXkGX7", 0), ROOT, "i"),
     ((1, "W7XhooU1Hsw7E", 0), ROOT, "s")],
    [((1, " f ", 0), ROOT, HIDE),
     ((2, " z ", 0), (1, " f ", 0), " "),
     ((2, " f ", 0), ROOT, "l"),
     ((2, " a ", 0), (1, " f ", 0), "v")],
    [((1, " f ", 0), ROOT, HIDE),
     ((2, " f ", 0), ROOT, HIDE),
     ((3, " a ", 0), (2, " f ", 0), "c"),
     ((2, " z ", 0), (1, " f ", 0), "r")],
]


def rand_node(ct, rng, site_ids, value=None):
    """list_test.cljc:15-29"""
    site = rng.choice(site_ids)
    cause = rng.choice(list(ct["nodes"].keys()))
    yarn = ct["yarns"].get(site)
    ts = 1 + max(cause[0], yarn[-1][0][0] if yarn else 0)
    return R.new_node(ts, site, cause, rng.choice(SIMPLE_VALUES) if value is None else value)


def random_history(rng, steps, nsites=5):
    """Grow a list by ``steps`` rand-node inserts; returns (nodes, final ct)."""
    sites = [R.new_site_id(rng) for _ in range(nsites)]
    ct = R.new_list_ct(rng=rng)
    nodes = []
    for _ in range(steps):
        nd = rand_node(ct, rng, sites)
        ct = R.insert(R.list_weave, ct, nd)
        nodes.append(nd)
    return nodes, ct


PROSE = ("Hereupon Legrand arose, with a grave and stately air, and brought me the beetle\n"
         "from a glass case in which it was enclosed. It was a beautiful scarabaeus, and, at\n"
         "that time, unknown to naturalists—of course a great prize in a scientific point\n"
         "of view. There were two round black spots near one extremity of the back, and a\n"
         "long one near the other. The scales were exceedingly hard and glossy, with all the\n"
         "appearance of burnished gold. The weight of the insect was very remarkable, and,\n"
         "taking all things into consideration, I could hardly blame Jupiter for his opinion\n"
         "respecting it.").split(" ")


def rand_phrase(rng):
    """list_test.cljc:127-130"""
    t = 2 + rng.randrange(6)
    d = max(rng.randrange(len(PROSE)) - t, 0)
    return " ".join(PROSE[d:d + t])


def rand_weave_of_phrases(rng, n_phrases=3):
    """list_test.cljc:132-155: each phrase typed by a new site, starting at ts 2
    caused by root, each char caused by the site's previous char."""
    phrases = [f" <{rand_phrase(rng)}> " for _ in range(n_phrases)]
    ct = R.new_list_ct(rng=rng)
    nodes = []
    for ph in phrases:
        site = R.new_site_id(rng)
        for ch in ph:
            yarn = ct["yarns"].get(site)
            cause = yarn[-1] if yarn else None
            nd = R.new_node(1 + (cause[0][0] if cause else 1), site,
                            cause[0] if cause else ROOT, ch)
            ct = R.insert(R.list_weave, ct, nd)
            nodes.append(nd)
    return ct, nodes, phrases


def stress_history(rng, n, nsites=8, p_special=0.2, p_hide_of_hide=0.2, p_conj=0.1,
                   p_chain=0.6, tx_chain=0.0):
    """A lamport-valid random list history (nodes incl. root, creation order).

    Causes: the site's previous node (p_chain), the current last weave node
    conj-style (p_conj, list.cljc:40 -- makes 'dirty' documents), else uniform.
    Specials: hides/h.hides/h.shows, a fraction caused by other specials.
    tx_chain: probability that a node continues the previous node's tx
    (same ts and site, tx-index + 1, caused by it).
    """
    sites = [R.new_site_id(rng) for _ in range(nsites)]
    nodes = [R.ROOT_NODE]
    clock = {s: 0 for s in sites}
    last = {s: None for s in sites}
    specials = []
    w = [R.ROOT_NODE]  # only to find the conj-style last weave node (incremental weave)
    for _ in range(n):
        prev = nodes[-1]
        if tx_chain and len(nodes) > 1 and rng.random() < tx_chain:
            (ts, site, tx) = prev[0]
            nd = ((ts, site, tx + 1), prev[0], rng.choice("abcdefg"))
        else:
            site = rng.choice(sites)
            r = rng.random()
            if r < p_special:
                if specials and rng.random() < p_hide_of_hide:
                    cause = rng.choice(specials)
                else:
                    cause = rng.choice(nodes)[0]
                value = rng.choice([HIDE, HIDE, H_HIDE, H_SHOW])
            else:
                value = rng.choice("abcdefghijklmnopqrstuvwxyz ")
                q = rng.random()
                if q < p_conj:
                    cause = w[-1][0]
                elif q < p_conj + p_chain and last[site] is not None:
                    cause = last[site]
                else:
                    cause = rng.choice(nodes)[0]
            cts = cause[0]
            ts = 1 + max(cts, clock[site])
            nd = ((ts, site, 0), cause, value)
        clock[nd[0][1]] = max(clock.get(nd[0][1], 0), nd[0][0])
        last[nd[0][1]] = nd[0]
        if R.is_special(nd[2]):
            specials.append(nd[0])
        nodes.append(nd)
        w = R.weave_node(w, nd)
    return nodes
