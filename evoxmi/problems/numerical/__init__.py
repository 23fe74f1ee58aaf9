from .classic import (
    Ackley, Griewank, Rastrigin, Rosenbrock, Schwefel, Sphere, Ellipsoid,
    ackley_func, griewank_func, rastrigin_func, rosenbrock_func, schwefel_func, sphere_func, ellipsoid_func,
)
