"""Drop-ins for comancpipeline.Tools native helpers (median_filter.medfilt, binFuncs)."""
