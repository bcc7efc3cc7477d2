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
               "ksim_encoder_pods", "ksim_encoder_node_order", "ksim_encoder_string"):
        assert f"C.{fn}(" in src["encoder.go"], fn
