"""stream-lib HyperLogLog(log2m=8).cardinality() for merging register sets on the broker side.

Register merge (`HyperLogLog.addAll`) is an element-wise max; the estimator uses alphaMM =
0.7213/(1+1.079/m)*m^2, linear counting m*ln(m/V) below 2.5*m, and Java Math.round (floor(x+0.5)).
"""
import math


def cardinality(registers):
    m = 256.0
    alpha_mm = (0.7213 / (1.0 + 1.079 / m)) * m * m
    s = 0.0
    zeros = 0.0
    for r in registers:
        r = int(r)
        s += 1.0 / (1 << r)
        if r == 0:
            zeros += 1.0
    est = alpha_mm * (1.0 / s)
    x = est
    if est <= 2.5 * m:
        x = m * math.log(m / zeros) if zeros > 0 else math.inf
    if math.isinf(x):
        return 9223372036854775807
    return int(math.floor(x + 0.5))
