// ref_driver.cpp — TEST INFRASTRUCTURE ONLY.
//
// A tiny command-line driver (our own code) linked against the reference's
// OWN host sources, compiled in place from /root/reference by oracle/Makefile
// into oracle/_ref/ref_driver:
//   src/core/utils/gaussians.cpp  (loadGaussiansFromPly, storeGaussianFromProperty)
//   src/core/scene/camera.cpp     (Camera: updateCameraMatrices, updateFrustumPlanes, orbit, zoom)
//   src/core/math/math.cpp        (MatVecMul_4D, MatMul_3D, GeMatMul, buildRotMatFromQuat, ...)
// It dumps their outputs as raw little-endian binaries so tests/golden/
// make_golden.py can turn them into fixtures that pin the oracle and the
// product's host helpers.  Nothing here is shipped or used at run time.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "camera.hpp"
#include "gaussians.hpp"
#include "math.hpp"

static void die(const char* m) {
    std::fprintf(stderr, "ref_driver: %s\n", m);
    std::exit(2);
}

static std::vector<float> read_floats(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) die("cannot open input");
    std::vector<float> v;
    float x;
    while (std::fread(&x, sizeof x, 1, f) == 1) v.push_back(x);
    std::fclose(f);
    return v;
}

// ply <in.ply> <out.bin>: n (int64) then 38 SoA arrays in gsr_types.h order.
static int cmd_ply(const char* in, const char* out) {
    std::vector<Gaussian> g = loadGaussiansFromPly(in);
    const int64_t n = (int64_t)g.size();
    std::vector<float> soa((size_t)38 * (size_t)n);
    for (int64_t i = 0; i < n; i++) {
        const Gaussian& q = g[(size_t)i];
        float* a = soa.data();
        a[0 * n + i] = q.x; a[1 * n + i] = q.y; a[2 * n + i] = q.z;
        a[3 * n + i] = q.opacity;
        for (int c = 0; c < 3; c++) a[(4 + c) * n + i] = q.scale[c];
        for (int c = 0; c < 4; c++) a[(7 + c) * n + i] = q.rot[c];
        for (int c = 0; c < 27; c++) a[(11 + c) * n + i] = q.sh[c];
    }
    FILE* f = std::fopen(out, "wb");
    if (!f) die("cannot open output");
    std::fwrite(&n, sizeof n, 1, f);
    std::fwrite(soa.data(), sizeof(float), soa.size(), f);
    std::fclose(f);
    return 0;
}

// camera <out.bin> px py pz lx ly lz ux uy uz fov aspect near far [op a b]...
// op: 'o' = orbit(a, b), 'z' = zoom(a).  Writes the 484-byte Camera after
// setup (updateCameraMatrices + updateFrustumPlanes) and after each op.
static int cmd_camera(int argc, char** argv) {
    if (argc < 15) die("camera: need 13 numbers");
    FILE* f = std::fopen(argv[2], "wb");
    if (!f) die("cannot open output");
    float v[13];
    for (int i = 0; i < 13; i++) v[i] = std::strtof(argv[3 + i], nullptr);
    Camera cam;
    cam.setPosition(v);
    cam.setLookAt(v + 3);
    cam.w_up[0] = v[6]; cam.w_up[1] = v[7]; cam.w_up[2] = v[8];
    cam.setFovY(v[9]);
    cam.setAspectRatio(v[10]);
    cam.setClippingPlanes(v[11], v[12]);
    cam.updateCameraMatrices();
    cam.updateFrustumPlanes();
    static_assert(sizeof(Camera) == 484, "Camera layout");
    std::fwrite(&cam, sizeof cam, 1, f);
    for (int i = 16; i + 2 < argc + 1 && i < argc; i += 3) {
        const char op = argv[i][0];
        const float a = std::strtof(argv[i + 1], nullptr);
        const float b = (i + 2 < argc) ? std::strtof(argv[i + 2], nullptr) : 0.0f;
        if (op == 'o') cam.orbit(a, b);
        else if (op == 'z') cam.zoom(a);
        else die("camera: bad op");
        std::fwrite(&cam, sizeof cam, 1, f);
    }
    std::fclose(f);
    return 0;
}

// chain <in.bin> <out.bin>: records of 21 floats (quat[4], scale[3], XYZ[3],
// fx, fy, r_cam[9]) -> Sigma2D[4] before pixel scaling, computed with the
// reference's math.cpp primitives in the order of render.cu:655-682.
static int cmd_chain(const char* in, const char* out) {
    std::vector<float> v = read_floats(in);
    const size_t nrec = v.size() / 21;
    FILE* f = std::fopen(out, "wb");
    if (!f) die("cannot open output");
    for (size_t r = 0; r < nrec; r++) {
        const float* q = &v[r * 21];
        float quat[4] = {q[0], q[1], q[2], q[3]};
        float scale[3] = {q[4], q[5], q[6]};
        const float X = q[7], Y = q[8], Z = q[9], fx = q[10], fy = q[11];
        float r_cam[9], r_cam_T[9];
        for (int i = 0; i < 9; i++) r_cam[i] = q[12 + i];
        transpose3x3(r_cam, r_cam_T);
        float jac[6], jacT[6], R[9], RT[9], S[9], tmp[9], cov[9], s2[4];
        jac[0] = fx / Z; jac[1] = 0.0f;
        jac[2] = -fx * X / (Z * Z); jac[3] = 0.0f;
        jac[4] = fy / Z; jac[5] = -fy * Y / (Z * Z);
        jacT[0] = jac[0]; jacT[1] = jac[3]; jacT[2] = jac[1];
        jacT[3] = jac[4]; jacT[4] = jac[2]; jacT[5] = jac[5];
        buildRotMatFromQuat(quat, R);
        transpose3x3(R, RT);
        buildDiagonalMatrix(scale, S);
        MatMul_3D(R, S, tmp);
        MatMul_3D(tmp, S, R);
        MatMul_3D(R, RT, cov);
        MatMul_3D(r_cam, cov, tmp);
        MatMul_3D(tmp, r_cam_T, cov);
        GeMatMul(jac, cov, 2, 3, 3, tmp);
        GeMatMul(tmp, jacT, 2, 2, 3, s2);
        std::fwrite(s2, sizeof(float), 4, f);
    }
    std::fclose(f);
    return 0;
}

// project <in.bin> <out.bin>: V[16], P[16], then xyz triples -> tmp[4], ndc[4]
// with MatVecMul_4D and the divisions of render.cu:545-548.
static int cmd_project(const char* in, const char* out) {
    std::vector<float> v = read_floats(in);
    if (v.size() < 32) die("project: short input");
    FILE* f = std::fopen(out, "wb");
    if (!f) die("cannot open output");
    for (size_t p = 32; p + 3 <= v.size(); p += 3) {
        float old_xyz[4] = {v[p], v[p + 1], v[p + 2], 1.0f};
        float tmp[4], nw[4];
        MatVecMul_4D(&v[0], old_xyz, tmp);
        MatVecMul_4D(&v[16], tmp, nw);
        nw[0] = nw[0] / nw[3];
        nw[1] = nw[1] / nw[3];
        nw[2] = nw[2] / nw[3];
        std::fwrite(tmp, sizeof(float), 4, f);
        std::fwrite(nw, sizeof(float), 4, f);
    }
    std::fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) die("usage: ref_driver ply|camera|chain|project ...");
    const std::string c = argv[1];
    if (c == "ply" && argc == 4) return cmd_ply(argv[2], argv[3]);
    if (c == "camera") return cmd_camera(argc, argv);
    if (c == "chain" && argc == 4) return cmd_chain(argv[2], argv[3]);
    if (c == "project" && argc == 4) return cmd_project(argv[2], argv[3]);
    die("bad command");
    return 2;
}
