"""Parameter grids restated from the reference's own tests
(dpf/distributed_point_function_test.cc), shared by the oracle tests and the
GPU API tests.  Value types use the oracle's tuple notation."""
from oracle import make_uint128

M32 = 4294967291                    # 2**32 - 5
M64 = 18446744073709551557          # 2**64 - 59
M80 = make_uint128(65535, 18446744073709551551)  # 2**80 - 65

# IncrementalDpfTest instantiations (test.cc:665-897): (levels, alphas, betas, level_steps)
ONE_LEVEL_ELEMENT_SIZES = [([(ld, bits)], [0, 1, 15], [[1], [100], [255]], [1])
                           for ld in (4, 10) for bits in (8, 16, 32, 64, 128)]
ONE_LEVEL_DOMAIN_SIZES = [([(ld, bits)], [0], [[1], [100], [255]], [1])
                          for bits in (8, 64, 128) for ld in range(10)]
TWO_LEVELS = [([(5, b), (10, b)], [0, 1, 2, 100, 1023], [[1, 2], [80, 90], [255, 255]], [1, 2])
              for b in (8, 16, 32, 64, 128)] + \
             [([(0, b), (10, 128)], [0, 1, 2, 100, 1023], [[1, 2], [80, 90], [255, 255]], [1, 2])
              for b in (8, 16, 32, 64, 128)]
THREE_LEVELS = [([(5, b), (10, b), (15, b)], [0, 1], [[1, 2, 3]], [1, 2])
                for b in (8, 16, 32, 64, 128)] + [
    ([(5, 8), (10, 16), (15, 32)], [0, 1], [[1, 2, 3]], [1, 2]),
    ([(4, 8), (5, 8), (6, 8)], [0, 1], [[1, 2, 3]], [1, 2]),
    ([(3, 16), (4, 16), (5, 16)], [0, 1], [[1, 2, 3]], [1, 2]),
    ([(2, 32), (3, 32), (4, 32)], [0, 1], [[1, 2, 3]], [1, 2]),
    ([(1, 64), (2, 64), (3, 64)], [0, 1], [[1, 2, 3]], [1, 2]),
    ([(0, 128), (1, 128), (2, 128)], [0, 1], [[1, 2, 3]], [1, 2]),
]
MAX_DOMAIN = ([(i, 64) for i in range(129)], [make_uint128(23, 42)], [[1234567] * 129],
              [1, 2, 3, 5, 7])

# DpfEvaluationTypes (test.cc:940-966), evaluated at log_domain 10, alpha 23,
# security_parameter 48, beta = all leaves 42.
EVALUATION_TYPES = [
    ("tuple", [("int", 8)]),
    ("tuple", [("int", 32)]),
    ("tuple", [("int", 128)]),
    ("tuple", [("int", 32), ("int", 32)]),
    ("tuple", [("int", 32), ("int", 64)]),
    ("tuple", [("int", 64), ("int", 64)]),
    ("tuple", [("int", 8), ("int", 16), ("int", 32), ("int", 64)]),
    ("tuple", [("int", 32)] * 4),
    ("tuple", [("int", 32), ("tuple", [("int", 32), ("int", 32)]), ("int", 32)]),
    ("tuple", [("int", 32), ("int", 128)]),
    ("intmodn", 32, M32),
    ("tuple", [("intmodn", 32, M32)]),
    ("tuple", [("int", 32), ("intmodn", 32, M32)]),
    ("tuple", [("int", 128), ("intmodn", 32, M32)]),
    ("tuple", [("intmodn", 32, M32), ("tuple", [("intmodn", 32, M32)])]),
    ("tuple", [("intmodn", 32, M32)] * 5),
    ("tuple", [("intmodn", 64, M64)] * 2),
    ("tuple", [("intmodn", 128, M80)] * 2),
    ("xor", 8),
    ("xor", 128),
    ("tuple", [("xor", 32), ("int", 128)]),
]
