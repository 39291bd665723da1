"""factormodeling_amd -- MI355X-native engine for the FactorModeling factor-panel hot path.

Drop-in modules (same names/signatures as the reference):
    factormodeling_amd.operations, .factor_selector, .factor_selection_methods,
    .composite_factor
Device-tensor layer:  factormodeling_amd.engine
Date-sharded multi-GPU driver:  factormodeling_amd.shard
"""
__version__ = "0.1.0"
