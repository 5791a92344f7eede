"""Reference-compatible namespace: ``from comapreduce_amd import Analysis`` then
``getattr(Analysis, name)`` for the TOML ``processes`` list exactly as
run_average.py:46-48 does with ``comancpipeline.Analysis``."""
from ..pipeline.running import Runner, PipelineFunction, set_logging  # noqa: F401
from ..pipeline.datahandling import HDF5Data, COMAPLevel1, COMAPLevel2, RepointEdges  # noqa: F401
from ..stages.level1 import (MeasureSystemTemperature, AtmosphereRemoval,  # noqa: F401
                             Level1AveragingGainCorrection, Level1Averaging, CheckLevel1File,
                             AssignLevel1Data)
from ..stages.statistics import Spikes, NoiseStatistics  # noqa: F401,E402
from ..stages.level2 import Level2FitPowerSpectrum  # noqa: F401,E402

STAGES = ('CheckLevel1File', 'AssignLevel1Data', 'MeasureSystemTemperature', 'AtmosphereRemoval',
          'Level1AveragingGainCorrection', 'Level1Averaging', 'Level2FitPowerSpectrum', 'Spikes',
          'NoiseStatistics')
