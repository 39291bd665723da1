"""factormodeling_amd -- MI355X-native engine for the FactorModeling factor-panel hot path.

Drop-in modules (same names/signatures as the reference):
    factormodeling_amd.operations, .factor_selector, .factor_selection_methods,
    .composite_factor, .portfolio_simulation, .multi_manager
    (factormodeling_amd/dropin/ puts them on sys.path under the reference's module names)
Device-tensor layer:  factormodeling_amd.engine (ctypes over libfmx.so, include/fmx.h)
Benchmark step and date-sharded multi-GPU driver:  factormodeling_amd.pipeline
    (ShardedPanel, run_step; exchanges through factormodeling_amd.comm)
CSV <-> panel I/O:  factormodeling_amd.csv_io (libfmx_io.so, include/fmx_io.h)
"""
__version__ = "0.1.0"
