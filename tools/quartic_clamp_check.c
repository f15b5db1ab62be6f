/* Exhaustive check behind the OneBlob forward's clamp shortcut (csrc/encodings.hip wrapped_cdf):
 * quartic_cdf (common_device.h:905-912) evaluated with the kernel's op sequence (explicit fmaf,
 * -ffp-contract=off) returns exactly 1.0f for every fp32 u >= T and exactly 0.0f for every u <= -T.
 * Prints the smallest such power-of-two-fraction T found and verifies it over all floats up to 2^20.
 *   gcc -O2 -ffp-contract=off -o /tmp/qc tools/quartic_clamp_check.c -lm && /tmp/qc */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float poly(float u) {
	const float u2 = u * u;
	const float u4 = u2 * u2;
	float p = fmaf(-(2.0f / 3.0f), u2, 1.0f);
	p = fmaf(1.0f / 5.0f, u4, p);
	return fmaxf(0.0f, fminf(1.0f, fmaf((15.0f / 16.0f) * u, p, 0.5f)));
}

static float f_of(uint32_t b) { float f; memcpy(&f, &b, 4); return f; }
static uint32_t b_of(float f) { uint32_t b; memcpy(&b, &f, 4); return b; }

int main(void) {
	/* largest u in [1, 2^20] whose result is not exactly 1 (resp. -u not exactly 0) */
	float last_hi = 0.0f, last_lo = 0.0f;
	for (uint32_t b = b_of(1.0f); b <= b_of(1048576.0f); ++b) {
		const float u = f_of(b);
		if (poly(u) != 1.0f) last_hi = u;
		if (poly(-u) != 0.0f) last_lo = u;
	}
	printf("last u with poly(u) != 1: %.9g   last u with poly(-u) != 0: %.9g\n", last_hi, last_lo);
	const float T = 1.0625f;
	int ok = last_hi < T && last_lo < T;
	printf("T = %.9g: %s\n", T, ok ? "OK" : "FAIL");
	return ok ? 0 : 1;
}
