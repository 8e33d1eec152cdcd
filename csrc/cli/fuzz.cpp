// `dmlc-fuzz`: mutation fuzzing of the parsers that read untrusted bytes,
// built with AddressSanitizer + UndefinedBehaviorSanitizer
// (build/bin/dmlc-fuzz-asan, tools/build.py; tests/test_fuzz_cpu.py):
//   * decode_jpeg          (query images, SDFS payloads: csrc/runtime/jpeg.cpp)
//   * decode_message       (membership UDP datagrams: csrc/control/membership.cpp)
//   * read_job / read_job_delta / read_directory (leader RPC payloads)
// Any out-of-bounds access or UB aborts the process under the sanitizers;
// parse errors are expected and caught.
//
// usage: dmlc-fuzz [--iters N] [--seed S] <seed jpeg files...>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "../control/membership.h"
#include "../control/sdfs.h"
#include "../runtime/jpeg.h"
#include "../serve/job.h"

using namespace dmlc;
using namespace dmlc::ctl;

namespace {

std::string mutate(const std::string& in, std::mt19937_64& rng) {
  std::string s = in;
  const int ops = 1 + (int)(rng() % 8);
  for (int k = 0; k < ops; ++k) {
    const size_t n = s.size();
    switch (rng() % 7) {
      case 0:  // bit flip
        if (n) s[rng() % n] ^= (char)(1 << (rng() % 8));
        break;
      case 1:  // interesting byte
        if (n) {
          static const unsigned char v[] = {0x00, 0xFF, 0x7F, 0x80, 0x01, 0xD8, 0xDA, 0xC0, 0xC4, 0xDB, 0xDD};
          s[rng() % n] = (char)v[rng() % sizeof(v)];
        }
        break;
      case 2:  // truncate
        if (n) s.resize(rng() % n);
        break;
      case 3:  // duplicate a chunk
        if (n > 2) {
          const size_t a = rng() % n, len = 1 + rng() % std::min<size_t>(n - a, 512);
          s.insert(rng() % n, s.substr(a, len));
        }
        break;
      case 4:  // erase a chunk
        if (n > 2) {
          const size_t a = rng() % n;
          s.erase(a, 1 + rng() % std::min<size_t>(n - a, 64));
        }
        break;
      case 5:  // big-endian 16-bit length field overwrite
        if (n > 2) {
          const size_t a = rng() % (n - 1);
          const uint16_t v = (uint16_t)(rng() % 3 == 0 ? 0xFFFF : rng() % 70000);
          s[a] = (char)(v >> 8);
          s[a + 1] = (char)v;
        }
        break;
      default:  // little-endian 32-bit count overwrite
        if (n > 4) {
          const size_t a = rng() % (n - 3);
          const uint32_t v = rng() % 3 == 0 ? 0xFFFFFFFFu : (uint32_t)(rng() % 4096);
          std::memcpy(&s[a], &v, 4);
        }
        break;
    }
  }
  return s;
}

std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

}  // namespace

int main(int argc, char** argv) {
  long iters = 20000;
  uint64_t seed = 1;
  std::vector<std::string> jpegs;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "--iters" && i + 1 < argc) iters = std::stol(argv[++i]);
    else if (a == "--seed" && i + 1 < argc) seed = std::stoull(argv[++i]);
    else jpegs.push_back(slurp(argv[i]));
  }
  std::mt19937_64 rng(seed);

  // seeds for the message parsers: valid encodings
  std::vector<std::string> msgs;
  {
    Message m;
    m.type = MsgType::Ping;
    m.sender = Id{"127.0.0.1:8850", 1234567};
    for (int i = 0; i < 5; ++i)
      m.list[Id{"10.0.0." + std::to_string(i) + ":8850", 1000 + i}] = Membership{Status::Active, 99 + i};
    msgs.push_back(encode_message(m));
    m.type = MsgType::Join;
    m.list.clear();
    msgs.push_back(encode_message(m));
  }
  std::vector<std::string> rpcs;
  {
    Job j;
    j.model_name = "resnet18";
    for (int i = 0; i < 20; ++i) j.add_result(i % 3 == 0, 1000 + i, 5000 + i);
    j.assigned.push_back(Id{"127.0.0.1:8850", 1});
    Writer w;
    write_job(w, j);
    rpcs.push_back(w.take());
    Writer d;
    write_job_delta(d, j, 7);
    rpcs.push_back(d.take());
    Directory dir;
    dir["a.txt"][Id{"127.0.0.1:8850", 1}] = {1, 2, 3};
    Writer wd;
    write_directory(wd, dir);
    rpcs.push_back(wd.take());
  }

  long parsed = 0, rejected = 0;
  for (long it = 0; it < iters; ++it) {
    const int which = (int)(rng() % 10);
    try {
      if (which < 6 && !jpegs.empty()) {
        const std::string in = mutate(jpegs[rng() % jpegs.size()], rng);
        Image img = decode_jpeg((const uint8_t*)in.data(), in.size());
        if ((size_t)img.width * img.height * 3 != img.rgb.size()) std::abort();
      } else if (which < 8) {
        const std::string in = mutate(msgs[rng() % msgs.size()], rng);
        decode_message(in.data(), in.size());
      } else {
        const size_t k = rng() % rpcs.size();
        const std::string in = mutate(rpcs[k], rng);
        Reader r(in);
        if (k == 0) read_job(r);
        else if (k == 1) {
          Job j;
          j.model_name = "resnet18";
          j.durations_us.assign(7, 1);
          j.done_us.assign(7, 1);
          read_job_delta(r, j);
        } else {
          read_directory(r);
        }
      }
      ++parsed;
    } catch (const std::exception&) {
      ++rejected;
    }
  }
  std::printf("fuzz: %ld iterations, %ld parsed, %ld rejected\n", iters, parsed, rejected);
  return 0;
}
