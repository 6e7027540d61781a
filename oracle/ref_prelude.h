// ref_prelude.h — TEST INFRASTRUCTURE.  Forced include (-include) for
// compiling the reference's own host C++ unmodified with g++ on Linux
// (oracle/Makefile, target ref-host).  It only pulls in standard headers the
// MSVC build got transitively and removes glibc's M_PI macro, which collides
// with the reference's own `constexpr double M_PI` (MCPT/oclbasic.h:192).
// It defines nothing of the reference's.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#undef M_PI
