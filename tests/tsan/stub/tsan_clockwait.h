// Force-included into the TSan build only (Makefile): GCC 11's libtsan does not intercept
// pthread_cond_clockwait, which libstdc++ 11 uses for condition_variable::wait_for on the steady
// clock, so TSan would miss the mutex release inside those waits and report false double locks
// and races.  Without the macro libstdc++ waits through pthread_cond_timedwait (intercepted).
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
