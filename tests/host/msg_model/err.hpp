// Test stand-in for the one macro of libzmq's src/err.hpp the binding uses
// (errno_assert: abort with the errno text when the condition fails).
#ifndef ZMQG_TEST_ERR_MODEL_HPP
#define ZMQG_TEST_ERR_MODEL_HPP
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define errno_assert(x)                                                        \
    do {                                                                       \
        if (!(x)) {                                                            \
            fprintf (stderr, "%s (%s:%d)\n", strerror (errno), __FILE__,       \
                     __LINE__);                                                \
            abort ();                                                          \
        }                                                                      \
    } while (false)
#endif
