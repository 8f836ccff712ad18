// Environment switches for A/B timing and debugging.  They exist only in
// builds made with -DDCC_EXPERIMENTS (`make EXPERIMENTS=1`); the product
// library reads no environment variable, so no variable can change a
// decision or select a timing variant with wrong results.
#pragma once
#ifdef DCC_EXPERIMENTS
#include <cstdlib>
#define DCC_ENV(name) getenv(name)
#else
#define DCC_ENV(name) ((const char*)nullptr)
#endif
