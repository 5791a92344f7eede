"""Destriping map-maker (reference comancpipeline/MapMaking)."""
