from .classic import (
    Ackley, Griewank, Rastrigin, Rosenbrock, Schwefel, Sphere, Ellipsoid,
    ackley_func, griewank_func, rastrigin_func, rosenbrock_func, schwefel_func, sphere_func, ellipsoid_func,
)
from .cec2022 import (
    CEC2022TestSuit, CEC2022TestSuite, F1_CEC2022, F2_CEC2022, F3_CEC2022, F4_CEC2022, F5_CEC2022, F6_CEC2022,
    F7_CEC2022, F8_CEC2022, F9_CEC2022, F10_CEC2022, F11_CEC2022, F12_CEC2022, cec2022_data,
)
