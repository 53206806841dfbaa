/*
 * keys_oracle.c -- CPU restatement of the key-handling helpers around the
 * CURVE path.  TEST INFRASTRUCTURE ONLY: the
 * checker for the device kernels, never linked into the product.
 *
 *   oracle_z85_encode / oracle_z85_decode
 *       zmq_z85_encode / zmq_z85_decode, reference src/zmq_utils.cpp:100-180
 *       (encoder / decoder tables :58-96).  Pinned by the reference's own
 *       vectors (tests/test_base85.cpp, tests/test_sodium.cpp key pair).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

static const char z85_enc[86] = "0123456789abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ.-:+=^!/*?&<>()[]{}@%$#";

/* 0xff = not a digit; index = character - 32, as the reference's table */
static uint8_t z85_dec[96];
static int z85_ready;

static void z85_init(void)
{
    if (z85_ready)
        return;
    memset(z85_dec, 0xff, sizeof z85_dec);
    for (int i = 0; i < 85; ++i)
        z85_dec[(uint8_t) z85_enc[i] - 32] = (uint8_t) i;
    z85_ready = 1;
}

/* 0, or EINVAL (22) when size % 4 != 0 (nothing written) */
EXPORT int oracle_z85_encode(char *dest, const uint8_t *data, uint64_t size)
{
    if (size % 4 != 0)
        return 22;
    uint64_t c = 0;
    for (uint64_t b = 0; b < size; b += 4) {
        uint32_t v = ((uint32_t) data[b] << 24) | ((uint32_t) data[b + 1] << 16) | ((uint32_t) data[b + 2] << 8) |
                     data[b + 3];
        uint32_t div = 85u * 85u * 85u * 85u;
        while (div) {
            dest[c++] = z85_enc[v / div % 85u];
            div /= 85u;
        }
    }
    dest[c] = 0;
    return 0;
}

/* 0, or EINVAL (22); `len` is strlen(string).  Groups before an invalid one
 * are written, as the reference's loop writes each group as it completes. */
EXPORT int oracle_z85_decode(uint8_t *dest, const char *string, uint64_t len)
{
    z85_init();
    if (len < 5 || len % 5 != 0)
        return 22;
    uint64_t byte_nbr = 0, char_nbr = 0;
    uint32_t value = 0;
    while (char_nbr < len) {
        if (UINT32_MAX / 85 < value)
            return 22;
        value *= 85;
        const uint8_t index = (uint8_t) ((uint8_t) string[char_nbr++] - 32);
        if (index >= sizeof z85_dec)
            return 22;
        const uint32_t summand = z85_dec[index];
        if (summand == 0xff || summand > UINT32_MAX - value)
            return 22;
        value += summand;
        if (char_nbr % 5 == 0) {
            dest[byte_nbr++] = (uint8_t) (value >> 24);
            dest[byte_nbr++] = (uint8_t) (value >> 16);
            dest[byte_nbr++] = (uint8_t) (value >> 8);
            dest[byte_nbr++] = (uint8_t) value;
            value = 0;
        }
    }
    return 0;
}
