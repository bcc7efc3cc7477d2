"""Restated result-store tests (simulator/scheduler/plugin/resultstore/store_test.go).

Same inputs and expected strings as the Go tests:
  * AddScoreResult: raw score + finalScore = raw x weight      (store_test.go:282-443)
  * AddNormalizedScoreResult overwrites finalScore             (store_test.go:445-578)
  * AddStoredResultToPod annotation JSON shapes                (store_test.go:580-848)
"""
import json

from ksim import resultstore as rs
from ksim.resultstore import Store, go_json


def test_add_score_result_applies_weight():
    s = Store({"plugin1": 2})
    s.add_score_result("default", "pod1", "node1", "plugin1", 10)
    r = s.results["default/pod1"]
    assert r.score == {"node1": {"plugin1": "10"}}
    assert r.final_score == {"node1": {"plugin1": "20"}}


def test_add_score_result_second_plugin_same_node():
    s = Store({"plugin2": 2})
    s.add_score_result("default", "pod1", "node1", "plugin1", 10)   # weight 0 for plugin1
    s.results["default/pod1"].final_score["node1"]["plugin1"] = "30"
    s.add_score_result("default", "pod1", "node1", "plugin2", 10)
    r = s.results["default/pod1"]
    assert r.final_score == {"node1": {"plugin1": "30", "plugin2": "20"}}
    assert r.score == {"node1": {"plugin1": "10", "plugin2": "10"}}


def test_add_normalized_score_result_overwrites_final():
    s = Store({"plugin1": 2})
    s.add_score_result("default", "pod1", "node0", "plugin1", 10)
    s.add_normalized_score_result("default", "pod1", "node0", "plugin1", 45)
    s.add_normalized_score_result("default", "pod1", "node1", "plugin1", 10)
    r = s.results["default/pod1"]
    assert r.score == {"node0": {"plugin1": "10"}}
    assert r.final_score == {"node0": {"plugin1": "90"}, "node1": {"plugin1": "20"}}


def test_add_stored_result_to_pod_full():
    s = Store({"plugin1": 2})
    ns, pod = "default", "pod1"
    s.add_selected_node(ns, pod, "node")
    s.add_pre_score_result(ns, pod, "plugin1", "preScore")
    s.add_pre_filter_result(ns, pod, "plugin1", "preFilterStatus", ["node2", "node1"])
    s.add_permit_result(ns, pod, "plugin1", "permit", "1s")
    s.add_reserve_result(ns, pod, "plugin1", "reserve")
    s.add_pre_bind_result(ns, pod, "plugin1", "prebind")
    s.add_bind_result(ns, pod, "plugin1", "bind")
    for n in ("node0", "node1"):
        s.add_filter_result(ns, pod, n, "plugin1", rs.PASSED_FILTER_MESSAGE)
        s.add_score_result(ns, pod, n, "plugin1", 10)
    s.add_post_filter_result(ns, pod, "node0", "plugin1", ["node0", "node1"])
    ann = {}
    s.add_stored_result_to_pod(ns, pod, ann)
    assert ann[rs.SELECTED_NODE] == "node"
    assert ann[rs.PRESCORE_RESULT] == '{"plugin1":"preScore"}'
    assert ann[rs.PREFILTER_RESULT] == '{"plugin1":["node1","node2"]}'
    assert ann[rs.PREFILTER_STATUS_RESULT] == '{"plugin1":"preFilterStatus"}'
    assert ann[rs.PERMIT_STATUS_RESULT] == '{"plugin1":"permit"}'
    assert ann[rs.PERMIT_TIMEOUT_RESULT] == '{"plugin1":"1s"}'
    assert ann[rs.RESERVE_RESULT] == '{"plugin1":"reserve"}'
    assert ann[rs.PREBIND_RESULT] == '{"plugin1":"prebind"}'
    assert ann[rs.BIND_RESULT] == '{"plugin1":"bind"}'
    assert ann[rs.FILTER_RESULT] == '{"node0":{"plugin1":"passed"},"node1":{"plugin1":"passed"}}'
    assert ann[rs.SCORE_RESULT] == '{"node0":{"plugin1":"10"},"node1":{"plugin1":"10"}}'
    assert ann[rs.FINALSCORE_RESULT] == '{"node0":{"plugin1":"20"},"node1":{"plugin1":"20"}}'
    assert ann[rs.POSTFILTER_RESULT] == '{"node0":{"plugin1":"preemption victim"},"node1":{}}'


def test_add_stored_result_to_pod_nothing_stored():
    s = Store({})
    ann = {}
    s.add_stored_result_to_pod("default", "pod1", ann)
    assert ann == {}


def test_add_stored_result_to_pod_partial_and_existing_keys_kept():
    s = Store({})
    s.add_filter_result("default", "pod1", "node0", "plugin1", "passed")
    ann = {rs.SCORE_RESULT: "keep-me"}
    s.add_stored_result_to_pod("default", "pod1", ann)
    assert ann[rs.SCORE_RESULT] == "keep-me"
    assert ann[rs.FINALSCORE_RESULT] == "{}"
    assert ann[rs.SELECTED_NODE] == ""
    for k in (rs.POSTFILTER_RESULT, rs.PRESCORE_RESULT, rs.PREFILTER_RESULT, rs.PREFILTER_STATUS_RESULT,
              rs.PERMIT_STATUS_RESULT, rs.PERMIT_TIMEOUT_RESULT, rs.RESERVE_RESULT, rs.PREBIND_RESULT,
              rs.BIND_RESULT):
        assert ann[k] == "{}"


def test_go_json_escapes_like_encoding_json():
    assert go_json({"b": "<x&y>", "a": "1"}) == '{"a":"1","b":"\\u003cx\\u0026y\\u003e"}'
    assert json.loads(go_json({"n": {"p": "node(s) had untolerated taint {a: b}"}}))


def test_delete_data():
    s = Store({})
    s.add_filter_result("default", "pod1", "node0", "plugin1", "passed")
    s.delete_data("default", "pod1")
    assert s.results == {}
