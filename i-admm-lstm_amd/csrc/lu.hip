// Stage II batched LU (models/lu.py) — placeholder translation unit; kernels land below.
#include "common.h"
