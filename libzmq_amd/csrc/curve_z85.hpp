// curve_z85.hpp -- batched Z85 (ZeroMQ RFC 32) key codec kernels, SURVEY.md
// section 8f row 4.  Semantics of zmq_z85_encode / zmq_z85_decode
// (reference src/zmq_utils.cpp:100-180), one item per thread: CURVE keys are
// 32 bytes / 40 characters, so a batch is many small independent items (the
// public keys of thousands of connections, or ZAP key lists).
//
// Encode: size % 4 != 0 -> EINVAL and nothing written; otherwise
// size * 5 / 4 characters and a terminating NUL.  Each 4-byte group is a
// big-endian value written as 5 base-85 digits, most significant first.
// Decode: len < 5 or len % 5 != 0 -> EINVAL and nothing written; otherwise
// groups are decoded in order and written as they complete, and the first
// invalid character or value above 0xffffffff stops the item with EINVAL
// (the groups before it are already written, as in the reference's loop).
// `len` plays strlen's part: a NUL byte inside it is an invalid character.
#pragma once

#include <errno.h>
#include <stdint.h>

namespace zmqg {

// "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#"
// (src/zmq_utils.cpp:58-62), as 85 characters
__constant__ const char z85_digits[86] =
    "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";

// Digit value of character c, 0xff if c is not a Z85 digit.
__device__ __forceinline__ uint32_t z85_value(uint32_t c)
{
    if (c >= '0' && c <= '9')
        return c - '0';
    if (c >= 'a' && c <= 'z')
        return c - 'a' + 10;
    if (c >= 'A' && c <= 'Z')
        return c - 'A' + 36;
    switch (c) {
    case '.': return 62;
    case '-': return 63;
    case ':': return 64;
    case '+': return 65;
    case '=': return 66;
    case '^': return 67;
    case '!': return 68;
    case '/': return 69;
    case '*': return 70;
    case '?': return 71;
    case '&': return 72;
    case '<': return 73;
    case '>': return 74;
    case '(': return 75;
    case ')': return 76;
    case '[': return 77;
    case ']': return 78;
    case '{': return 79;
    case '}': return 80;
    case '@': return 81;
    case '%': return 82;
    case '$': return 83;
    case '#': return 84;
    default: return 0xffu;
    }
}

__global__ __launch_bounds__(256) void k_z85_encode(uint32_t n, const uint64_t *__restrict__ in_off,
                                                    const uint32_t *__restrict__ len, const uint8_t *__restrict__ in,
                                                    const uint64_t *__restrict__ out_off, char *__restrict__ out,
                                                    int32_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t size = len[i];
    if (size % 4u != 0u) {
        status[i] = EINVAL;
        return;
    }
    const uint8_t *p = in + in_off[i];
    char *d = out + out_off[i];
    for (uint32_t g = 0; g < size / 4u; ++g) {
        uint32_t v = ((uint32_t) p[4 * g] << 24) | ((uint32_t) p[4 * g + 1] << 16) | ((uint32_t) p[4 * g + 2] << 8) |
                     (uint32_t) p[4 * g + 3];
        char c[5];
#pragma unroll
        for (int k = 4; k >= 0; --k) {
            c[k] = z85_digits[v % 85u];
            v /= 85u;
        }
#pragma unroll
        for (int k = 0; k < 5; ++k)
            d[5 * g + k] = c[k];
    }
    d[size / 4u * 5u] = 0;
    status[i] = 0;
}

__global__ __launch_bounds__(256) void k_z85_decode(uint32_t n, const uint64_t *__restrict__ in_off,
                                                    const uint32_t *__restrict__ len, const char *__restrict__ in,
                                                    const uint64_t *__restrict__ out_off, uint8_t *__restrict__ out,
                                                    int32_t *__restrict__ status)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t size = len[i];
    if (size < 5u || size % 5u != 0u) {
        status[i] = EINVAL;
        return;
    }
    const uint8_t *p = (const uint8_t *) in + in_off[i];
    uint8_t *d = out + out_off[i];
    for (uint32_t g = 0; g < size / 5u; ++g) {
        uint32_t v = 0;
        for (int k = 0; k < 5; ++k) {
            // src/zmq_utils.cpp:148-163: overflow before the multiply, then
            // the digit, then overflow of the sum
            if (0xffffffffu / 85u < v) {
                status[i] = EINVAL;
                return;
            }
            v *= 85u;
            const uint32_t s = z85_value(p[5 * g + k]);
            if (s == 0xffu || s > 0xffffffffu - v) {
                status[i] = EINVAL;
                return;
            }
            v += s;
        }
        d[4 * g] = (uint8_t) (v >> 24);
        d[4 * g + 1] = (uint8_t) (v >> 16);
        d[4 * g + 2] = (uint8_t) (v >> 8);
        d[4 * g + 3] = (uint8_t) v;
    }
    status[i] = 0;
}

} // namespace zmqg
