/* byte / 255.0f against pt_shading.h u8_unit's form: x * fl(1/255), then one
 * fma correction -- correctly rounded (the IEEE division's value) for every
 * byte 0..255; exits 1 on any mismatch.  Test tool (tests/test_libmf.py). */
#include <math.h>
#include <stdio.h>
#include <string.h>

int main(void) {
    int bad = 0;
    const volatile float r = 1.0f / 255.0f;
    for (unsigned b = 0; b < 256; b++) {
        const volatile float x = (float)b;
        const volatile float div = x / 255.0f;
        const volatile float q = x * r;
        const float u = fmaf(fmaf(-q, 255.0f, x), r, q);
        if (memcmp((const void*)&div, &u, 4) != 0) bad++;
    }
    printf("u8_unit mismatches: %d of 256\n", bad);
    return bad != 0;
}
