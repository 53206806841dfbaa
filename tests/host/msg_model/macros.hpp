// Test stand-in for the one macro of libzmq's src/macros.hpp the binding
// uses: a class that can be neither copied nor moved.
#ifndef ZMQG_TEST_MACROS_MODEL_HPP
#define ZMQG_TEST_MACROS_MODEL_HPP
#define ZMQ_NON_COPYABLE_NOR_MOVABLE(classname)                                \
  public:                                                                      \
    classname (const classname &) = delete;                                    \
    classname &operator= (const classname &) = delete;
#endif
