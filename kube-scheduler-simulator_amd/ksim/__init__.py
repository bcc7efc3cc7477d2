"""ksim — MI355X-native engine for the kube-scheduler-simulator scheduling cycle.

Host-side package: ABI mirror (abi), object model (model), snapshot encoder
(encode), profile conversion (profile), synthetic configs (gen), the engine
binding (engine) and the simulator-side result recording (resultstore,
wrapped).  The compute path is libksim_engine.so (HIP, gfx950).
"""
__all__ = ["abi", "model", "encode", "profile", "gen"]
