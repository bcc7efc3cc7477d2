"""The Go side of the drop-in (integration/go/engine, not compiled here: no Go
toolchain) stays in step with include/ksim_engine.h: the binding's ABIVersion
is the header's KSIM_ABI_VERSION, and every C.ksim_* / C.KSIM_* name the Go
sources use is declared by the header."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "integration", "go", "engine")
HDR = open(os.path.join(ROOT, "include", "ksim_engine.h")).read()


def _go_sources():
    return {f: open(os.path.join(GO, f)).read() for f in sorted(os.listdir(GO)) if f.endswith(".go")}


def test_abi_version_matches_header():
    hv = int(re.search(r"#define KSIM_ABI_VERSION (\d+)", HDR).group(1))
    gv = int(re.search(r"const ABIVersion = (\d+)", _go_sources()["engine.go"]).group(1))
    assert gv == hv, f"integration/go/engine/engine.go ABIVersion {gv} != header {hv}"


def test_go_names_declared_in_header():
    declared_fns = set(re.findall(r"\b(ksim_\w+)\s*\(", HDR))
    declared_types = set(re.findall(r"}\s*(ksim_\w+);", HDR)) | set(re.findall(r"typedef struct (ksim_\w+)", HDR))
    declared_macros = set(re.findall(r"#define (KSIM_\w+)", HDR))
    missing = []
    for f, src in _go_sources().items():
        for name in set(re.findall(r"\bC\.(ksim_\w+)", src)):
            if name not in declared_fns and name not in declared_types:
                missing.append((f, name))
        for name in set(re.findall(r"\bC\.(KSIM_\w+)", src)):
            if name not in declared_macros:
                missing.append((f, name))
    assert not missing, missing


def test_framework_entry_points_bound():
    """The framework-driven calls the engine-backed plugins need are bound."""
    src = "\n".join(_go_sources().values())
    for fn in ("ksim_fw_prefilter", "ksim_fw_score", "ksim_fw_normalize", "ksim_assume", "ksim_forget",
               "ksim_preempt", "ksim_preempt_nominated", "ksim_fw_filter_nominated"):
        assert f"C.{fn}(" in src, fn


def test_native_encoder_implements_encoder():
    """integration/go/engine/encoder.go NativeEncoder has every method of the
    Encoder interface the engine-backed plugins call (plugins.go), and drives
    the native snapshot encoder of the header."""
    src = _go_sources()
    iface = re.search(r"type Encoder interface \{(.*?)\n\}", src["plugins.go"], re.S).group(1)
    methods = set(re.findall(r"^\t([A-Z]\w*)\(", iface, re.M))
    impl = set(re.findall(r"^func \(n \*NativeEncoder\) ([A-Z]\w*)\(", src["encoder.go"], re.M))
    assert methods and methods <= impl, methods - impl
    for fn in ("ksim_encoder_create", "ksim_encode_nodes", "ksim_encode_pods", "ksim_encoder_cluster",
               "ksim_encoder_pods", "ksim_encoder_string"):
        assert f"C.{fn}(" in src["encoder.go"], fn


def test_native_encoder_applies_deltas():
    """ABI 11: the Go encoder follows informer events with the encoder's delta
    calls (ksim/fwsnapshot.py is its Python mirror, tests/test_fw_snapshot.py
    and tests/test_gpu_fw_snapshot.py run that mirror): node events through
    ksim_encoder_update_nodes + ksim_upsert_nodes, bound pods through
    ksim_assume / ksim_forget + ksim_encoder_bind / _unbind, the framework's
    Reserve / Unreserve through Encoder.Assume / Forget, and no per-cycle walk
    of the NodeInfos' pods."""
    src = _go_sources()
    enc, plg = src["encoder.go"], src["plugins.go"]
    for fn in ("ksim_encoder_update_nodes", "ksim_encoder_old_pos", "ksim_encoder_bind", "ksim_encoder_unbind"):
        assert f"C.{fn}(" in enc, fn
    assert "e.UpsertNodes(" in enc and "e.Assume(" in enc and "e.Forget(" in enc
    assert "func (n *NativeEncoder) Handlers()" in enc
    assert "fed.Handlers()" in plg and ".Informer().AddEventHandler(" in plg
    assert "pr.Enc.Assume(" in plg and "pr.Enc.Forget(" in plg and "pr.Enc.BoundTable(" in plg
    snap = re.search(r"func \(n \*NativeEncoder\) Snapshot\(.*?\n}\n", enc, re.S).group(0)
    # the framework's NodeInfos are read once, at the first cycle (the whole snapshot)
    assert snap.count("NodeInfos().List()") == 1 and "if !n.encoded" in snap


def test_spread_defaulting_defaults_to_system():
    """PodTopologySpreadArgs.defaultingType defaults to System upstream; the
    Go encoder's zero value must mean the same, "None" opts out."""
    enc = _go_sources()["encoder.go"]
    m = re.search(r'case "", "System":[^\n]*\n\s*opts.spread_defaults = C.KSIM_SPREAD_DEFAULTS_SYSTEM', enc)
    assert m, "empty SpreadDefaulting must select KSIM_SPREAD_DEFAULTS_SYSTEM"
    assert 'case "None":' in enc
