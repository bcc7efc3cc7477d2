"""Result store: the simulator's per-pod result maps and their annotations.

A one-to-one mirror of simulator/scheduler/plugin/resultstore/store.go
(Store.Add* at store.go:418-603, AddStoredResultToPod at store.go:129-190,
applyWeightOnScore at store.go:499-502) with the annotation keys of
simulator/scheduler/plugin/annotation/annotation.go:3-30.  Values are the same
strings the Go store writes; JSON is encoded the way Go's encoding/json does
(sorted map keys, compact, HTML-escaped).
"""
from __future__ import annotations

import json
import threading
from typing import Dict, List, Optional

# annotation.go
PREFILTER_STATUS_RESULT = "scheduler-simulator/prefilter-result-status"
PREFILTER_RESULT = "scheduler-simulator/prefilter-result"
FILTER_RESULT = "scheduler-simulator/filter-result"
POSTFILTER_RESULT = "scheduler-simulator/postfilter-result"
PRESCORE_RESULT = "scheduler-simulator/prescore-result"
SCORE_RESULT = "scheduler-simulator/score-result"
FINALSCORE_RESULT = "scheduler-simulator/finalscore-result"
RESERVE_RESULT = "scheduler-simulator/reserve-result"
PERMIT_STATUS_RESULT = "scheduler-simulator/permit-result"
PERMIT_TIMEOUT_RESULT = "scheduler-simulator/permit-result-timeout"
PREBIND_RESULT = "scheduler-simulator/prebind-result"
BIND_RESULT = "scheduler-simulator/bind-result"
SELECTED_NODE = "scheduler-simulator/selected-node"

# store.go:27-36
PASSED_FILTER_MESSAGE = "passed"
SUCCESS_MESSAGE = "success"
WAIT_MESSAGE = "wait"
POST_FILTER_NOMINATED_MESSAGE = "preemption victim"


def go_json(obj) -> str:
    """encoding/json.Marshal for maps/slices/strings: sorted keys, no spaces,
    <, >, & and U+2028/U+2029 escaped."""
    s = json.dumps(obj, sort_keys=True, separators=(",", ":"), ensure_ascii=False)
    return (s.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
            .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))


class _Result:
    __slots__ = ("selected_node", "pre_score", "score", "final_score", "pre_filter_status",
                 "pre_filter_result", "filter", "post_filter", "permit", "permit_timeout",
                 "reserve", "prebind", "bind")

    def __init__(self):
        self.selected_node = ""
        self.pre_score: Dict[str, str] = {}
        self.score: Dict[str, Dict[str, str]] = {}
        self.final_score: Dict[str, Dict[str, str]] = {}
        self.pre_filter_status: Dict[str, str] = {}
        self.pre_filter_result: Dict[str, List[str]] = {}
        self.filter: Dict[str, Dict[str, str]] = {}
        self.post_filter: Dict[str, Dict[str, str]] = {}
        self.permit: Dict[str, str] = {}
        self.permit_timeout: Dict[str, str] = {}
        self.reserve: Dict[str, str] = {}
        self.prebind: Dict[str, str] = {}
        self.bind: Dict[str, str] = {}


class Store:
    """resultstore.Store."""

    def __init__(self, score_plugin_weight: Dict[str, int]):
        self.mu = threading.Lock()
        self.results: Dict[str, _Result] = {}
        self.score_plugin_weight = dict(score_plugin_weight)

    @staticmethod
    def _key(namespace: str, pod_name: str) -> str:
        return namespace + "/" + pod_name

    def _get(self, ns: str, name: str) -> _Result:
        k = self._key(ns, name)
        r = self.results.get(k)
        if r is None:
            r = self.results[k] = _Result()
        return r

    # --- Add* (store.go:418-603) ----------------------------------------------
    def add_filter_result(self, ns, pod, node, plugin, reason):
        with self.mu:
            self._get(ns, pod).filter.setdefault(node, {})[plugin] = reason

    def add_post_filter_result(self, ns, pod, nominated_node, plugin, node_names):
        with self.mu:
            r = self._get(ns, pod)
            for n in node_names:
                r.post_filter.setdefault(n, {})
                if n == nominated_node:
                    r.post_filter[n][plugin] = POST_FILTER_NOMINATED_MESSAGE

    def add_score_result(self, ns, pod, node, plugin, score: int):
        with self.mu:
            r = self._get(ns, pod)
            r.score.setdefault(node, {})[plugin] = str(int(score))
            self._add_normalized(r, node, plugin, score)

    def add_normalized_score_result(self, ns, pod, node, plugin, score: int):
        with self.mu:
            self._add_normalized(self._get(ns, pod), node, plugin, score)

    def _add_normalized(self, r: _Result, node, plugin, score):
        r.final_score.setdefault(node, {})[plugin] = str(self.apply_weight_on_score(plugin, score))

    def apply_weight_on_score(self, plugin: str, score: int) -> int:
        return int(score) * int(self.score_plugin_weight.get(plugin, 0))

    def delete_data(self, ns, pod):
        with self.mu:
            self.results.pop(self._key(ns, pod), None)

    def add_pre_filter_result(self, ns, pod, plugin, reason, node_names: Optional[List[str]] = None):
        with self.mu:
            r = self._get(ns, pod)
            r.pre_filter_status[plugin] = reason
            if node_names is not None:
                r.pre_filter_result[plugin] = sorted(node_names)   # sets.String.List() is sorted

    def add_pre_score_result(self, ns, pod, plugin, reason):
        with self.mu:
            self._get(ns, pod).pre_score[plugin] = reason

    def add_permit_result(self, ns, pod, plugin, status, timeout: str):
        with self.mu:
            r = self._get(ns, pod)
            r.permit[plugin] = status
            r.permit_timeout[plugin] = timeout

    def add_selected_node(self, ns, pod, node):
        with self.mu:
            self._get(ns, pod).selected_node = node

    def add_reserve_result(self, ns, pod, plugin, status):
        with self.mu:
            self._get(ns, pod).reserve[plugin] = status

    def add_bind_result(self, ns, pod, plugin, status):
        with self.mu:
            self._get(ns, pod).bind[plugin] = status

    def add_pre_bind_result(self, ns, pod, plugin, status):
        with self.mu:
            self._get(ns, pod).prebind[plugin] = status

    # --- AddStoredResultToPod (store.go:129-190) -------------------------------
    def add_stored_result_to_pod(self, namespace: str, name: str, annotations: Dict[str, str]) -> None:
        """Writes every result map into ``annotations`` (skipping keys already present)."""
        with self.mu:
            r = self.results.get(self._key(namespace, name))
            if r is None:
                return
            a = annotations

            def put(key, value):
                if key not in a:
                    a[key] = value

            put(PREFILTER_RESULT, go_json(r.pre_filter_result))
            put(PREFILTER_STATUS_RESULT, go_json(r.pre_filter_status))
            put(FILTER_RESULT, go_json(r.filter))
            put(POSTFILTER_RESULT, go_json(r.post_filter))
            put(PRESCORE_RESULT, go_json(r.pre_score))
            put(SCORE_RESULT, go_json(r.score))
            put(FINALSCORE_RESULT, go_json(r.final_score))
            put(RESERVE_RESULT, go_json(r.reserve))
            put(PERMIT_TIMEOUT_RESULT, go_json(r.permit_timeout))
            put(PERMIT_STATUS_RESULT, go_json(r.permit))
            put(PREBIND_RESULT, go_json(r.prebind))
            put(BIND_RESULT, go_json(r.bind))
            put(SELECTED_NODE, r.selected_node)
