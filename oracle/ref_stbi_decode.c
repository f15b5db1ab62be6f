// ref_stbi_decode.c -- TEST INFRASTRUCTURE. Decodes a JPEG with the reference's own vendored
// stb_image (dependencies/stbi/stb_image.h, compiled as it lies under /root/reference; the decoder
// behind the sample's load_image -> load_stbi, stbi_wrapper.cpp:37-44) and writes the 8-bit pixels as
// a binary PGM (1 channel) or PPM (3 channels). stbi_loadf, which the sample calls, is
// pow(u8 / 255, 2.2) of exactly these values (stb_image.h:1838-1849), so the 8-bit decode pins the
// sample's training image; consumers apply the gamma themselves.
// Used by tools/make_albert_full.py to build tests/golden/albert_full.png and the PSNR of the
// reference's own renders data/readme/{100,1000}.jpg. Build: `make -C oracle ref` (-> oracle/_ref/).
//
//   stbi_decode <in.jpg> <out.pgm|out.ppm> <channels: 1|3>
#define STB_IMAGE_IMPLEMENTATION
#include <stbi/stb_image.h>

#include <stdio.h>
#include <stdlib.h>

int main(int argc, char** argv) {
	if (argc != 4) {
		fprintf(stderr, "usage: %s in.jpg out.pnm channels(1|3)\n", argv[0]);
		return 2;
	}
	const int req = atoi(argv[3]);
	if (req != 1 && req != 3) {
		fprintf(stderr, "channels must be 1 or 3\n");
		return 2;
	}
	int w = 0, h = 0, n = 0;
	unsigned char* px = stbi_load(argv[1], &w, &h, &n, req);
	if (!px) {
		fprintf(stderr, "stbi_load failed: %s\n", stbi_failure_reason());
		return 1;
	}
	FILE* f = fopen(argv[2], "wb");
	if (!f) {
		stbi_image_free(px);
		return 1;
	}
	fprintf(f, "%s\n%d %d\n255\n", req == 1 ? "P5" : "P6", w, h);
	const size_t bytes = (size_t)w * h * req;
	const int ok = fwrite(px, 1, bytes, f) == bytes;
	fclose(f);
	stbi_image_free(px);
	printf("%s: %dx%d, %d source channel(s) -> %d\n", argv[1], w, h, n, req);
	return ok ? 0 : 1;
}
