"""The fast forms equal the literal fold at full size, on the CPU (no GPU).

SURVEY F4/F5 say the linked fold and the effective-tree preorder equal the
reference's literal weave-node fold (shared.cljc:225-241 over list.cljc:26-28)
whenever every cause is present and older.  Here that is checked on the first
64 full config-2 documents of the bench workload (50,001 nodes each, ~40%
dirty: a non-special node caused by a special one), weave order and rendered
bits, so the GPU tests that compare full-size batches with METHOD_EFF rest on
a literal-pinned restatement.
"""
import numpy as np

import oracle
from cause_amd import gen
from tests import fullsize as F


def test_literal_equals_linked_equals_eff_on_64_full_config2_documents():
    off, idk, ck, kd = gen.generate(gen.CONFIG2, 0, 64)
    dirty = F.dirty_docs(off, idk, ck, kd)
    assert 16 <= dirty.sum() <= 48, dirty.sum()
    pl, vl, sl = oracle.batch_lists(off, idk, ck, kd, method=oracle.METHOD_LITERAL)
    assert not sl.any()
    for m in (oracle.METHOD_LINKED, oracle.METHOD_EFF):
        p, v, s = oracle.batch_lists(off, idk, ck, kd, method=m)
        assert not s.any()
        assert np.array_equal(p, pl), m
        assert np.array_equal(v, vl), m
    # the literal fold's rendered bits are hide? on its own weave (list.cljc:48-55)
    for d in (0, 1, int(np.flatnonzero(dirty)[0])):
        a, b = int(off[d]), int(off[d + 1])
        lit = oracle.list_visible(idk[a:b], ck[a:b], kd[a:b], pl[a:b])
        assert np.array_equal(lit, vl[a:b])
