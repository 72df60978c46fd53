from tianshou_amd.utils.statistics import (DeviceRunningMeanStd, DeviceScalarRMS,
                                           RunningMeanStd)

__all__ = ["RunningMeanStd", "DeviceRunningMeanStd", "DeviceScalarRMS"]
