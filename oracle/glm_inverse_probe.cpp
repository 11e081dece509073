// TEST INFRASTRUCTURE.  glm::inverse(mat4) as the reference's own build
// compiles it (g++ -std=gnu++20 -O3 -march=native, the glm vendored under
// /root/reference), for checking pt_mat4_inverse (pt_bvh.cpp) bit for bit:
//   g++ -std=gnu++20 -O3 -march=native -fno-math-errno -fno-trapping-math \
//       -I/root/reference oracle/glm_inverse_probe.cpp -o oracle/_ref/glm_inverse_probe
//   oracle/_ref/glm_inverse_probe in.bin out.bin   (16 floats per matrix, column-major)
// Built by oracle/Makefile (`make -C oracle ref`); tests/golden/gen_golden.py records its
// output as tests/golden/mat4_inverse.npz.
#include <cstdio>
#include <glm/glm.hpp>
int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* in = fopen(argv[1], "rb");
    FILE* out = fopen(argv[2], "wb");
    if (!in || !out) return 2;
    glm::mat4 m;
    while (fread(&m[0][0], 4, 16, in) == 16) {
        const glm::mat4 inv = glm::inverse(m);
        fwrite(&inv[0][0], 4, 16, out);
    }
    fclose(in);
    fclose(out);
    return 0;
}
