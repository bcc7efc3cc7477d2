"""NetworkBandwidth, the simulator's out-of-tree plugin — host side.

simulator/scheduler/plugin/networkbandwidth/plugin.go registers it next to the
in-tree plugins (simulator/scheduler/config/plugin.go:214-221,266-273,279-284);
a profile enables it for Filter and / or Score.  The string work (annotation
lookup, resource.ParseQuantity) happens here once per node and pod; the device
only compares and subtracts integers:

* node: the limit annotation -> KSIM_NODE_NB_LIMIT (present) /
  KSIM_NODE_NB_LIMIT_BAD (does not parse), ``nb_limit`` in milli-units;
  ``nb_alloc`` = getNodeAllocatedAmount over the bound pods (plugin.go:104-123:
  the ingress and egress *request* annotations, unparsable ones skipped);
* pod: ``nb_req`` = the Filter request (plugin.go:65-90: each request
  annotation falling back to kubernetes.io/{ingress,egress}-bandwidth),
  KSIM_POD_NB_{INGRESS,EGRESS}_BAD when one does not parse; ``nb_add`` = the
  pod's share of a node's allocated amount once bound.

Quantities are held in milli-units, where int64 Quantity arithmetic is exact;
a quantity with a finer fraction or out of that range is refused
(EncodeError), not rounded.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from fractions import Fraction
from typing import Dict, Optional, Tuple

from . import abi

INGRESS_BANDWIDTH = "kubernetes.io/ingress-bandwidth"   # plugin.go:21
EGRESS_BANDWIDTH = "kubernetes.io/egress-bandwidth"     # plugin.go:22


@dataclass
class NetworkBandwidthArgs:
    """NetworkBandwidthArgs with New's defaults (plugin.go:200-204,222-228)."""
    node_limit_annotation: str = "node.kubernetes.io/network-limit"
    egress_request_annotation: str = "kubernetes.io/egress-request"
    ingress_request_annotation: str = "kubernetes.io/ingress-request"

    @classmethod
    def from_config(cls, args: Optional[dict]) -> "NetworkBandwidthArgs":
        """DecodeInto over the defaults: fields the document omits keep them."""
        a, d = cls(), args or {}
        if "nodeLimitAnnotation" in d:
            a.node_limit_annotation = str(d["nodeLimitAnnotation"] or "")
        if "egressRequestAnnotation" in d:
            a.egress_request_annotation = str(d["egressRequestAnnotation"] or "")
        if "ingressRequestAnnotation" in d:
            a.ingress_request_annotation = str(d["ingressRequestAnnotation"] or "")
        return a


class QuantityError(ValueError):
    """A parsable quantity the engine cannot hold exactly in milli-units."""


_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1,
        "k": 10 ** 3, "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}
# resource.ParseQuantity's grammar: <signedNumber><suffix>, no surrounding space
_QRE = re.compile(r"([+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+))(Ki|Mi|Gi|Ti|Pi|Ei|[numkMGTPE]|[eE][+-]?[0-9]+)?")
_I64 = 2 ** 63


def milli(s: str) -> Optional[int]:
    """resource.ParseQuantity(s) in milli-units; None when it does not parse."""
    m = _QRE.fullmatch(s)
    if not m:
        return None
    v = Fraction(m.group(1))
    suf = m.group(2) or ""
    if suf in _BIN:
        v *= _BIN[suf]
    elif suf in _DEC:
        v *= _DEC[suf]
    else:
        v *= Fraction(10) ** int(suf[1:])
    v *= 1000
    if v.denominator != 1:
        raise QuantityError(f"quantity {s!r} is finer than 1m")
    if not -_I64 < v.numerator < _I64 // 1024:      # headroom for sums of many pods
        raise QuantityError(f"quantity {s!r} out of the engine's range")
    return int(v)


def node_limit(annotations: Dict[str, str], args: NetworkBandwidthArgs) -> Tuple[int, int]:
    """(KSIM_NODE_NB_* flags, limit in milli-units)."""
    if args.node_limit_annotation not in annotations:
        return 0, 0
    q = milli(annotations[args.node_limit_annotation])
    if q is None:
        return abi.NODE_NB_LIMIT | abi.NODE_NB_LIMIT_BAD, 0
    return abi.NODE_NB_LIMIT, q


def pod_request(annotations: Dict[str, str], args: NetworkBandwidthArgs) -> Tuple[int, int]:
    """(KSIM_POD_NB_* flags, Filter request in milli-units), plugin.go:65-90."""
    total, flags = 0, 0
    for key, fallback, bad in ((args.ingress_request_annotation, INGRESS_BANDWIDTH, abi.POD_NB_INGRESS_BAD),
                               (args.egress_request_annotation, EGRESS_BANDWIDTH, abi.POD_NB_EGRESS_BAD)):
        s = annotations.get(key, annotations.get(fallback))
        if s is None:
            continue
        q = milli(s)
        if q is None:
            flags |= bad
        else:
            total += q
    return flags, total


def pod_allocated(annotations: Dict[str, str], args: NetworkBandwidthArgs) -> int:
    """The pod's share of getNodeAllocatedAmount (plugin.go:104-123), milli-units."""
    total = 0
    for key in (args.ingress_request_annotation, args.egress_request_annotation):
        if key in annotations:
            q = milli(annotations[key])
            if q is not None:
                total += q
    return total


# messages the wrapper records (plugin.go:56,60,75,87,93,98)
def filter_message(detail: int, node: str, pod: str, args: NetworkBandwidthArgs) -> str:
    if detail == abi.NB_INSUFFICIENT:
        return f"Node {node} does not have enough network bandwidth capacity to schedule pod"
    if detail == abi.NB_NO_LIMIT:
        return f"Node {node} does not have {args.node_limit_annotation} annotation present"
    if detail == abi.NB_LIMIT_BAD:
        return f"Node {node} has an incorrect quantity in {args.node_limit_annotation} annotation present"
    if detail == abi.NB_INGRESS_BAD:
        return f"Could not parse quantity from pod {pod} {args.ingress_request_annotation} annotations"
    if detail == abi.NB_EGRESS_BAD:
        return f"Could not parse quantity from pod {pod} {args.egress_request_annotation} annotations"
    if detail == abi.NB_NO_REQUEST:
        return (f"Pod {pod} does not have network bandwidth request annotations set. "
                f"(Missing {args.ingress_request_annotation} or {args.egress_request_annotation})")
    raise ValueError(f"unknown NetworkBandwidth detail {detail}")
