"""Host-side pipeline: data model and stage runner (reference Analysis/{DataHandling,Running}.py)."""
from .datahandling import HDF5Data, COMAPLevel1, COMAPLevel2, RepointEdges, level1_from_dict  # noqa: F401
from .running import PipelineFunction, Runner, set_logging  # noqa: F401
