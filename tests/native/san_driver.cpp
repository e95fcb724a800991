// san_driver.cpp — host-code driver for the sanitizer builds (tools/run_sanitizers.sh; SURVEY §5,
// race detection). TEST INFRASTRUCTURE ONLY. It links the host-instrumented device plugin, front
// end and oracle (make SAN=...) and drives, on the host-only device (no GPU):
//   scenes  <file>...        every scene loader (.ecs command files, .xml, .obj/.mtl, Collada .dae
//                            through -fprCollada): parse, commit (BVH build, scene upload mirrors),
//                            export the frame blob and render a 16x16 thumbnail with the oracle
//   images  <file>...        the PNG / baseline-JPEG / PPM decoders (yrtDebugDecodeImage,
//                            rtNewImageFromFile) and the image writers (.jpg/.png/.ppm/.pfm)
//   fuzz <seed> <n> <file>...  n mutations of each file (byte flips, truncation, splices; seeded)
//                            fed to the matching loader: every one must load or fail cleanly
//   hub <rounds>             the shard hub's host phases from several threads (status exchange,
//                            slabs, a peer that never sends, a size mismatch) — the TSan build
// Exit status 0 when every step returned; sanitizer reports abort the process (halt_on_error).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/yrt_device.h"
#include "../../include/yrt_frontend.h"
#include "../../oracle/yrt_oracle.h"

static std::string ext_of(const std::string& f) {
  const size_t d = f.find_last_of('.');
  std::string e = d == std::string::npos ? "" : f.substr(d + 1);
  for (char& c : e) c = (char)tolower((unsigned char)c);
  return e;
}

static std::vector<uint8_t> read_file(const std::string& f) {
  std::ifstream in(f, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

static void write_file(const std::string& f, const std::vector<uint8_t>& b) {
  std::ofstream out(f, std::ios::binary);
  out.write((const char*)b.data(), (std::streamsize)b.size());
}

// One scene file through the front end on the host-only device; returns 0 when it loaded.
static int load_scene(YRTDevice dev, const std::string& f, bool render) {
  const std::string e = ext_of(f);
  std::vector<std::string> args;
  if (e == "ecs") args = {"-c", f};
  else if (e == "dae") args = {"-fprCollada", "-i", f};
  else args = {"-i", f};
  for (const char* a : {"-size", "16", "16", "-spp", "2", "-fb", "RGB_FLOAT32"}) args.push_back(a);
  std::vector<const char*> argv;
  for (const auto& a : args) argv.push_back(a.c_str());
  YRTSession s = yrtSessionCreate(dev, (int)argv.size(), argv.data());
  if (!s) return 1;
  YRTSessionInfo info;
  int rc = yrtSessionInfo(s, &info);
  if (rc == 0 && render) {
    YRTHandle cam = yrtSessionNumSceneCameras(s) > 0 ? yrtSessionSceneCamera(s, 0) : yrtSessionCamera(s, -1);
    const int64_t n = yrtExportFrame(dev, info.renderer, cam, info.scene, nullptr, 0);
    if (n > 0) {
      std::vector<uint8_t> blob((size_t)n);
      yrtExportFrame(dev, info.renderer, cam, info.scene, blob.data(), blob.size());
      std::vector<float> img(16 * 16 * 3, 0.f);
      OracleStats st;
      if (oracle_render(blob.data(), blob.size(), 16, 16, info.gamma, 0, 0, 16, 16, 2, img.data(), &st) != 0)
        rc = 2;
    }
  }
  yrtSessionDestroy(s);
  return rc;
}

static int load_image(YRTDevice dev, const std::string& f) {
  int w = 0, h = 0, c = 0;
  int rc = 0;
  const std::string e = ext_of(f);
  if (e == "png" || e == "jpg" || e == "jpeg") {
    // the decoder alone (0: decoded; the size comes back first), then into a buffer
    rc = yrtDebugDecodeImage(f.c_str(), &w, &h, &c, nullptr, 0) != 0;
    if (!rc) {
      std::vector<uint8_t> px((size_t)w * h * c);
      rc = yrtDebugDecodeImage(f.c_str(), &w, &h, &c, px.data(), px.size()) != 0;
    }
  }
  // rtNewImageFromFile: a file that fails to load becomes a 1x1 white image
  // (singleray_device.cpp:238-251), so only the decoders' status is reported
  YRTHandle im = yrtNewImageFromFile(dev, f.c_str());
  if (im) yrtDecRef(dev, im);
  return rc;
}

static int write_images(const std::string& dir) {
  const int W = 37, H = 23;
  std::vector<uint8_t> rgb8(W * H * 3);
  std::vector<float> rgbf(W * H * 3);
  for (int i = 0; i < W * H * 3; ++i) {
    rgb8[i] = (uint8_t)(i * 7);
    rgbf[i] = (float)(i % 97) / 31.f;
  }
  int rc = 0;
  for (const char* e : {"jpg", "png", "ppm"}) {
    const std::string f = dir + "/san_out." + e;
    rc |= yrtStoreImage(f.c_str(), W, H, 0, rgb8.data(), (size_t)W * 3, 90);
  }
  rc |= yrtStoreImage((dir + "/san_out.pfm").c_str(), W, H, 2, rgbf.data(), (size_t)W * 12, 0);
  for (int q : {1, 50, 100}) rc |= yrtStoreImage((dir + "/san_q.jpg").c_str(), W, H, 0, rgb8.data(), (size_t)W * 3, q);
  return rc;
}

// Seeded mutations of a file: flips, truncation, a zero run, a duplicated block.
static std::vector<uint8_t> mutate(const std::vector<uint8_t>& in, std::mt19937& rng) {
  std::vector<uint8_t> b = in;
  if (b.empty()) return b;
  std::uniform_int_distribution<size_t> pos(0, b.size() - 1);
  switch (rng() % 5) {
    case 0:
      for (int k = 0; k < 1 + (int)(rng() % 8); ++k) b[pos(rng)] ^= (uint8_t)(1u << (rng() % 8));
      break;
    case 1: b.resize(pos(rng)); break;
    case 2: {
      const size_t p = pos(rng), n = std::min<size_t>(b.size() - p, 1 + rng() % 64);
      std::memset(b.data() + p, (rng() & 1) ? 0xff : 0, n);
      break;
    }
    case 3: {
      const size_t p = pos(rng), n = std::min<size_t>(b.size() - p, 1 + rng() % 256);
      std::vector<uint8_t> blk(b.begin() + (long)p, b.begin() + (long)(p + n));
      b.insert(b.begin() + (long)pos(rng), blk.begin(), blk.end());
      break;
    }
    default:
      for (int k = 0; k < 4; ++k) b[pos(rng)] = (uint8_t)rng();
      break;
  }
  return b;
}

static int hub_rounds(int rounds) {
  int bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const int world = 2 + r % 3;
    YRTShardHub hub = yrtNewShardHub(world);
    // status exchange and slabs from `world` threads
    std::vector<int> st(world, -2);
    std::vector<std::thread> th;
    for (int k = 0; k < world; ++k) th.emplace_back([&, k] { st[k] = yrtShardHubStatus(hub, k, k == 1 ? 0 : 1, 10.0); });
    for (auto& t : th) t.join();
    th.clear();
    for (int k = 0; k < world; ++k) bad += st[k] != 0;
    std::vector<std::vector<uint8_t>> data(world, std::vector<uint8_t>(64));
    std::vector<uint8_t> recv((size_t)world * 64);
    std::vector<int> sl(world, -2);
    for (int k = 0; k < world; ++k) {
      std::memset(data[k].data(), k + 1, 64);
      th.emplace_back([&, k] {
        sl[k] = k == 0 ? yrtShardHubSlab(hub, 0, nullptr, 0, recv.data(), 64, 10.0)
                       : yrtShardHubSlab(hub, k, data[k].data(), 64, nullptr, 0, 10.0);
      });
    }
    for (auto& t : th) t.join();
    th.clear();
    for (int k = 0; k < world; ++k) bad += sl[k] != 0;
    for (int k = 1; k < world; ++k) bad += recv[(size_t)(k - 1) * 64] != (uint8_t)(k + 1);
    yrtDeleteShardHub(hub);
    // a peer that never sends: rank 0's receive ends at its deadline with an error
    hub = yrtNewShardHub(2);
    th.emplace_back([&] { st[0] = yrtShardHubStatus(hub, 0, 1, 5.0); });
    th.emplace_back([&] { st[1] = yrtShardHubStatus(hub, 1, 1, 5.0); });
    for (auto& t : th) t.join();
    th.clear();
    bad += yrtShardHubSlab(hub, 0, nullptr, 0, recv.data(), 16, 0.05) != -1;
    yrtDeleteShardHub(hub);
    // a slab of the wrong size is refused on both sides
    hub = yrtNewShardHub(2);
    th.emplace_back([&] { st[0] = yrtShardHubStatus(hub, 0, 1, 5.0); });
    th.emplace_back([&] { st[1] = yrtShardHubStatus(hub, 1, 1, 5.0); });
    for (auto& t : th) t.join();
    th.clear();
    std::vector<uint8_t> big(100, 7);
    th.emplace_back([&] { sl[0] = yrtShardHubSlab(hub, 0, nullptr, 0, recv.data(), 64, 5.0); });
    th.emplace_back([&] { sl[1] = yrtShardHubSlab(hub, 1, big.data(), big.size(), nullptr, 0, 5.0); });
    for (auto& t : th) t.join();
    bad += !(sl[0] == -1 || sl[1] == -1);
    yrtDeleteShardHub(hub);
  }
  return bad;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s scenes|images|fuzz|hub ...\n", argv[0]);
    return 2;
  }
  setvbuf(stdout, nullptr, _IOLBF, 0);  // progress lines reach the log as they happen
  const std::string mode = argv[1];
  if (mode == "hub") {
    const int bad = hub_rounds(argc > 2 ? atoi(argv[2]) : 4);
    std::printf("hub: %d unexpected results\n", bad);
    return bad ? 1 : 0;
  }
  YRTDevice dev = yrtNewDevice("host", 0, 0, nullptr);
  if (!dev) {
    std::fprintf(stderr, "no host device\n");
    return 1;
  }
  int rc = 0;
  if (mode == "scenes") {
    for (int i = 2; i < argc; ++i) {
      const int r = load_scene(dev, argv[i], true);
      std::printf("scene %-60s %s\n", argv[i], r ? "FAILED" : "ok");
      rc |= r;
    }
  } else if (mode == "images") {
    for (int i = 2; i < argc; ++i) {
      const int r = load_image(dev, argv[i]);
      std::printf("image %-60s %s\n", argv[i], r ? "FAILED" : "ok");
      rc |= r;
    }
    const char* tmp = getenv("TMPDIR");
    rc |= write_images(tmp ? tmp : "/tmp");
  } else if (mode == "fuzz" && argc > 4) {
    std::mt19937 rng((unsigned)atoi(argv[2]));
    const int n = atoi(argv[3]);
    const char* tmp = getenv("TMPDIR");
    for (int i = 4; i < argc; ++i) {
      const std::string f = argv[i], e = ext_of(f);
      const std::vector<uint8_t> orig = read_file(f);
      // the mutated copy keeps the extension (and, for scene files, the directory: relative
      // texture and .mtl references still resolve)
      const size_t slash = f.find_last_of('/');
      const bool scene = e == "ecs" || e == "xml" || e == "obj" || e == "dae" || e == "mtl";
      const std::string dir = scene && slash != std::string::npos ? f.substr(0, slash) : std::string(tmp ? tmp : "/tmp");
      const std::string mf = dir + "/_san_fuzz_" + std::to_string(i) + "." + e;
      int loaded = 0;
      for (int k = 0; k < n; ++k) {
        write_file(mf, mutate(orig, rng));
        if (e == "mtl") continue;  // reached through its .obj
        const int r = scene ? load_scene(dev, mf, false) : load_image(dev, mf);
        loaded += r == 0;
      }
      std::remove(mf.c_str());
      std::printf("fuzz %-60s %d mutations, %d loaded, the rest refused cleanly\n", f.c_str(), n, loaded);
    }
  } else {
    std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
    rc = 2;
  }
  yrtDeleteDevice(dev);
  return rc;
}
