"""The JVM twins (CauseWeave.java, list_gpu.clj) against include/causeweave.h,
read as text (no JDK here: tests/jvm_twins.py).  Round 4 showed how the twins
drift silently; these tests fail on a drifted constant, layout, offset or
binding and pass on the committed sources."""
import pytest

from tests import jvm_twins as J


def test_committed_twins_are_in_line():
    assert J.check_twins(*J.read_sources()) == []


def test_the_parsers_see_the_whole_contract():
    h, j, c = J.read_sources()
    hc = J.header_constants(h)
    assert hc["CW_STATUS_KEY_RANGE"] == 128 and hc["CW_KIND_ROOT"] == 4
    hs = J.header_structs(h)
    assert [f for f, *_ in hs["cw_list_batch"]][-1] == "site_bits"
    assert hs["cw_list_batch"][-1][3] == 52          # offset of site_bits
    assert hs["cw_map_result"][-1][3] == 56          # offset of status
    from cause_amd import abi

    assert set(J.header_functions(h)) == set(abi.header_functions())
    jh = J.java_handles(j)
    assert set(jh) == {"cw_ctx_create", "cw_ctx_destroy", "cw_last_error", "cw_weave_lists",
                       "cw_weave_lists_k128", "cw_weave_maps"}
    acc = J.java_segment_accesses(j)
    assert len(acc) >= 30 and {a[0] for a in acc} == set(J.LAYOUTS)


@pytest.mark.parametrize("old,new,what", [
    ("STATUS_DUP = 2", "STATUS_DUP = 4", "STATUS_DUP"),
    ("KIND_HSHOW = 3", "KIND_HSHOW = 2", "KIND_HSHOW"),
    ("STATUS_KEY_RANGE = 128;", "STATUS_KEY_RANGE = 256;", "STATUS_KEY_RANGE"),
    ('JAVA_INT.withName("ts_shift"), JAVA_INT.withName("site_shift")',
     'JAVA_INT.withName("site_shift"), JAVA_INT.withName("ts_shift")', "LIST_BATCH"),
    ("b.set(JAVA_INT, 52, siteBits)", "b.set(JAVA_INT, 56, siteBits)", "offset 56"),
    ("res.set(ADDRESS, 56, status)", "res.set(JAVA_INT, 56, status)", "JAVA_INT at offset 56"),
    ('FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_INT));\n  static final MethodHandle WEAVE_MAPS',
     'FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, JAVA_INT));\n  static final MethodHandle WEAVE_MAPS',
     "cw_weave_lists_k128"),
    ('h("cw_weave_maps"', 'h("cw_weave_map"', "cw_weave_map"),
])
def test_a_drifted_java_twin_fails(old, new, what):
    h, j, c = J.read_sources()
    assert old in j, old
    problems = J.check_twins(h, j.replace(old, new, 1), c)
    assert problems and any(what in p for p in problems), problems


@pytest.mark.parametrize("old,new,what", [
    ("CauseWeave/STATUS_KEY_RANGE", "CauseWeave/STATUS_KEYRANGE", "STATUS_KEYRANGE"),
    ("(.weavePerm r)", "(.weaveperm r)", ".weaveperm"),
    ("(.weaveMaps ^CauseWeave", "(.weaveMap ^CauseWeave", ".weaveMap"),
    ("CauseWeave$ListResult", "CauseWeave$ListResults", "ListResults"),
])
def test_a_drifted_clojure_twin_fails(old, new, what):
    h, j, c = J.read_sources()
    assert old in c, old
    problems = J.check_twins(h, j, c.replace(old, new))
    assert problems and any(what in p for p in problems), problems


def test_a_drifted_header_fails():
    h, j, c = J.read_sources()
    h2 = h.replace("CW_STATUS_WEFT = 1u << 6", "CW_STATUS_WEFT = 1u << 9")
    assert h2 != h
    assert any("STATUS_WEFT" in p for p in J.check_twins(h2, j, c))
