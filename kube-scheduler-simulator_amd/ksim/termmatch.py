"""Selector / affinity-term matching on the device.

Upstream PodTopologySpread and InterPodAffinity match their selectors and
terms against every existing pod in PreFilter / PreScore ([upstream]
podtopologyspread countPodsMatchSelector, interpodaffinity
getExistingAntiAffinityCounts / getIncomingAffinityAntiAffinityCounts /
processExistingPod; reached per pod through
simulator/scheduler/plugin/wrappedplugin.go:427-486).  ksim/topology.py keeps
the answers as count classes.  This module compiles the matchers of a
TopologyIndex into a ``ksim_match_problem`` and lets the engine answer it with
an int8 contraction on the matrix cores (csrc/ksim_match.hip):

  features      ("ns", name), ("kv", key, value), ("key", key) — only the ones
                some requirement names
  signature     the feature set of a (namespace, labels) pair
  requirement   In(k, V) / matchLabels k=v   positive over ("kv", k, v), v in V
                NotIn(k, V)                  negative over the same features
                Exists(k) / DoesNotExist(k)  positive / negative over ("key", k)
                namespace predicate          positive over ("ns", n), n in the set
                nil selector                 positive over no feature (never)
  matcher       AND of its requirements (a Matcher, or ("all", (Matcher, ..))
                for podMatchesAllAffinityTerms)

A requirement holds for a signature when (number of shared features > 0)
differs from its negative flag, which is exactly LabelSelector.matches on the
label map (model.py) and the namespace test of TopologyIndex.matches.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import abi


def _p(a: np.ndarray):
    return a.ctypes.data if a.size else None


class MatchProblem:
    """The matchers of a TopologyIndex as requirements over features, and a
    set of signatures as feature sets (numpy CSR arrays + the ctypes struct)."""

    def __init__(self, topo, matchers: Sequence, sigs: Sequence[tuple]):
        self.feat: Dict[tuple, int] = {}
        self.req_ids: Dict[Tuple[bool, frozenset], int] = {}
        self.req_neg: List[int] = []
        self.req_feats: List[List[int]] = []
        m_reqs: List[List[int]] = []
        for m in matchers:
            reqs: List[int] = []
            for sub in (m[1] if isinstance(m, tuple) and m and m[0] == "all" else (m,)):
                reqs.extend(self._matcher_reqs(topo, sub))
            m_reqs.append(reqs)
        self.n_matchers = len(matchers)
        self.n_words = (self.n_matchers + 31) // 32
        # signatures: (namespace, sorted label items) -> feature ids in the
        # vocabulary; signatures with the same features (labels no requirement
        # names differ) share one row of the contraction (sig_row)
        rows: Dict[tuple, int] = {}
        sig_feats = []
        self.sig_row = np.zeros(len(sigs), np.int32)
        for i, (ns, labels) in enumerate(sigs):
            f = []
            x = self.feat.get(("ns", ns))
            if x is not None:
                f.append(x)
            for k, v in labels:
                for key in (("kv", k, v), ("key", k)):
                    x = self.feat.get(key)
                    if x is not None:
                        f.append(x)
            t = tuple(sorted(f))
            r = rows.get(t)
            if r is None:
                r = rows[t] = len(sig_feats)
                sig_feats.append(list(t))
            self.sig_row[i] = r
        self.sig_off, self.sig_feat = _csr(sig_feats)
        self.req_off, self.req_feat = _csr(self.req_feats)
        self.neg = np.array(self.req_neg, np.uint8)
        self.m_off, self.m_req = _csr(m_reqs)
        self.n_sigs = len(sig_feats)                    # distinct feature sets (rows)
        self.pod_sig = np.zeros(0, np.int32)
        self.pod_node = np.zeros(0, np.int32)
        self.class_matcher = np.zeros(0, np.int32)
        self.n_nodes = 0

    def _fid(self, key: tuple) -> int:
        i = self.feat.get(key)
        if i is None:
            i = self.feat[key] = len(self.feat)
        return i

    def _req(self, neg: bool, keys) -> int:
        fs = frozenset(self._fid(k) for k in keys)
        rk = (neg, fs)
        r = self.req_ids.get(rk)
        if r is None:
            r = self.req_ids[rk] = len(self.req_neg)
            self.req_neg.append(1 if neg else 0)
            self.req_feats.append(sorted(fs))
        return r

    def _matcher_reqs(self, topo, m) -> List[int]:
        out = []
        if not m.all_namespaces:
            out.append(self._req(False, [("ns", n) for n in sorted(m.namespaces)]))
        if m.selector is None:
            out.append(self._req(False, []))
            return out
        match_labels, exprs = m.selector
        for k, v in match_labels:
            out.append(self._req(False, [("kv", k, v)]))
        for k, op, vals in exprs:
            if op in ("In", "NotIn"):
                out.append(self._req(op == "NotIn", [("kv", k, v) for v in vals]))
            elif op in ("Exists", "DoesNotExist"):
                out.append(self._req(op == "DoesNotExist", [("key", k)]))
            else:                                        # rejected by _validate_selector
                raise ValueError(f"selector operator {op}")
        return out

    def set_counts(self, pod_sig: np.ndarray, pod_node: np.ndarray, n_nodes: int, class_matcher: Sequence[int]):
        """Count classes to accumulate over bound pods (signature index into
        the constructor's ``sigs``, node)."""
        self.pod_sig = np.ascontiguousarray(self.sig_row[np.asarray(pod_sig, np.int64)], np.int32)
        self.pod_node = np.ascontiguousarray(pod_node, np.int32)
        self.class_matcher = np.ascontiguousarray(class_matcher, np.int32)
        self.n_nodes = int(n_nodes)

    def struct(self) -> abi.MatchProblem:
        s = abi.MatchProblem()
        s.n_sigs, s.n_feat, s.n_reqs, s.n_matchers = self.n_sigs, len(self.feat), len(self.req_neg), self.n_matchers
        s.sig_feat_off, s.sig_feat = _p(self.sig_off), _p(self.sig_feat)
        s.req_feat_off, s.req_feat = _p(self.req_off), _p(self.req_feat)
        s.req_neg, s.m_req_off, s.m_req = _p(self.neg), _p(self.m_off), _p(self.m_req)
        s.n_pods, s.n_nodes, s.n_classes = int(self.pod_sig.size), self.n_nodes, int(self.class_matcher.size)
        s.pod_sig, s.pod_node, s.class_matcher = _p(self.pod_sig), _p(self.pod_node), _p(self.class_matcher)
        return s


def _csr(rows: List[List[int]]) -> Tuple[np.ndarray, np.ndarray]:
    off = np.zeros(len(rows) + 1, np.int32)
    if rows:
        off[1:] = np.cumsum([len(r) for r in rows])
    flat = np.fromiter((x for r in rows for x in r), np.int32, int(off[-1]))
    return off, flat


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    """[rows][ceil(n/32)] u32 -> [rows][n] bool (bit m of a row's words)."""
    if n == 0:
        return np.zeros((words.shape[0], 0), bool)
    b = np.unpackbits(words.astype("<u4").view(np.uint8).reshape(words.shape[0], -1), axis=1, bitorder="little")
    return b[:, :n].astype(bool)


def expand_rows(mp: MatchProblem, hit: np.ndarray) -> np.ndarray:
    """[distinct feature sets][matchers] -> [constructor sigs][matchers]."""
    return hit[mp.sig_row]


class DeviceMatcher:
    """TopologyIndex.matcher backed by the engine (ksim_match_terms)."""

    def __init__(self, engine):
        self.engine = engine
        self.calls = 0

    def match(self, mp: MatchProblem):
        """-> (bool [n_sigs][n_matchers], int32 [n_classes][n_nodes])."""
        counts = np.zeros((mp.class_matcher.size, mp.n_nodes), np.int32) if mp.class_matcher.size else None
        bits = self.engine.match_terms(mp.struct(), mp.n_words, counts)
        self.calls += 1
        return expand_rows(mp, unpack_bits(bits, mp.n_matchers)), counts
