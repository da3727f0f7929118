"""Full-size parity against the reference's literal fold (METHOD_LITERAL:
weave-node clause for clause, shared.cljc:194-241 over list.cljc:26-28), not
against a restatement of it:

* 24 full config-2 documents (50,001 nodes each), 12 dirty and 12 clean
  (tests/fullsize.py), in one batch through the default pipeline -- order,
  rendered bits, counts, ::lamport-ts and yarns;
* config 1 in full (one list of 100,001 nodes, the giant-document path);
* the same 24 documents under the HBM walk and the radix front end.
"""
import numpy as np
import pytest

import oracle
from cause_amd import abi, gen
from tests import fullsize as F
from tests.test_gpu_parity import check_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mixed():
    return F.config2_mixed(12, 12)


@pytest.mark.parametrize("knobs", [{}, {"CW_FUSED": "0"}, {"CW_TOUR": "0"}, {"CW_FRONT": "0"}],
                         ids=["default", "separate", "hbm-walk", "radix"])
def test_config2_full_documents_vs_literal(mixed, knobs, monkeypatch):
    off, idk, ck, kd, dirty, lay = mixed
    assert len(dirty) == 24 and dirty.sum() == 12
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    with abi.Weaver(0) as w:
        res = check_batch(w, off, idk, ck, kd, lay, method=oracle.METHOD_LITERAL)
    assert not res.status.any()


def test_config1_full_vs_literal():
    off, idk, ck, kd = gen.generate(gen.CONFIG1, 0, 1)
    with abi.Weaver(0) as w:
        res = check_batch(w, off, idk, ck, kd, gen.CONFIG1.layout(), method=oracle.METHOD_LITERAL)
    assert not res.status.any()
