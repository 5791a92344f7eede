"""Pipeline stages (drop-ins for the reference Analysis stage classes)."""
from .level1 import (MeasureSystemTemperature, AtmosphereRemoval, Level1AveragingGainCorrection,  # noqa: F401
                     CheckLevel1File, AssignLevel1Data)
