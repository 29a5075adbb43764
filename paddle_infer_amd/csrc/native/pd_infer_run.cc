// Command-line driver of the native C++ predictor (no Python):
//   pd_infer_run <model.pdmodel> <model.pdiparams> [--gpu DEV] [--precision fp32|fp16|bf16]
//                [--graph] [--threads N] [--warmup W] [--repeat R] [--step-input NAME]
//                --input NAME DTYPE D0,D1,.. FILE.bin ...  --output-dir DIR
// Inputs are raw little-endian files; each fetch target is written to DIR/<index>.bin with its
// shape on stdout ("output <i> <name> <dtype> d0,d1,..") and the mean Run() time last.
// --step-input NAME: the int32 scalar input NAME advances by one before every Run after the
// first (a decode loop: fused_multi_transformer TimeStep over caches that stay resident).
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>

#include "paddle_inference_api.h"

using namespace paddle_infer;

static std::vector<int> parse_dims(const std::string& s) {
  std::vector<int> d;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, ','))
    if (!t.empty()) d.push_back(std::stoi(t));
  return d;
}

static std::string read_all(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: pd_infer_run model.pdmodel model.pdiparams [--gpu D] --input NAME DTYPE DIMS FILE ... --output-dir DIR\n";
    return 2;
  }
  try {
    Config cfg(argv[1], argv[2]);
    struct In { std::string name, dtype, file; std::vector<int> dims; };
    std::vector<In> ins;
    std::string outdir = ".";
    int repeat = 1, warmup = 0, gpu = -1;
    PrecisionType prec = PrecisionType::kFloat32;
    std::string step_input;
    for (int i = 3; i < argc; ++i) {
      const std::string a = argv[i];
      if (a == "--gpu") gpu = std::stoi(argv[++i]);
      else if (a == "--precision") {
        const std::string p = argv[++i];
        prec = p == "bf16" ? PrecisionType::kBf16 : p == "fp16" ? PrecisionType::kHalf : PrecisionType::kFloat32;
      } else if (a == "--step-input") step_input = argv[++i];
      else if (a == "--threads") cfg.SetCpuMathLibraryNumThreads(std::stoi(argv[++i]));
      else if (a == "--repeat") repeat = std::stoi(argv[++i]);
      else if (a == "--warmup") warmup = std::stoi(argv[++i]);
      else if (a == "--graph") cfg.EnableHipGraph(true);
      else if (a == "--output-dir") outdir = argv[++i];
      else if (a == "--input") {
        In in;
        in.name = argv[++i];
        in.dtype = argv[++i];
        in.dims = parse_dims(argv[++i]);
        in.file = argv[++i];
        ins.push_back(in);
      } else {
        std::cerr << "unknown argument " << a << "\n";
        return 2;
      }
    }
    if (gpu >= 0) cfg.EnableUseGpu(256, gpu, prec);
    auto pred = CreatePredictor(cfg);
    std::vector<std::string> raw;
    int32_t step0 = 0;
    for (auto& in : ins) {
      raw.push_back(read_all(in.file));
      auto h = pred->GetInputHandle(in.name);
      h->Reshape(in.dims);
      if (in.dtype == "float32") h->CopyFromCpu(reinterpret_cast<const float*>(raw.back().data()));
      else if (in.dtype == "int64") h->CopyFromCpu(reinterpret_cast<const int64_t*>(raw.back().data()));
      else if (in.dtype == "int32") h->CopyFromCpu(reinterpret_cast<const int32_t*>(raw.back().data()));
      else throw std::runtime_error("unsupported input dtype " + in.dtype);
      if (in.name == step_input) step0 = *reinterpret_cast<const int32_t*>(raw.back().data());
    }
    int runs = 0;
    auto advance = [&]() {
      if (step_input.empty() || runs++ == 0) return;
      const int32_t t = step0 + runs - 1;
      auto h = pred->GetInputHandle(step_input);
      h->Reshape({1});
      h->CopyFromCpu(&t);
    };
    for (int r = 0; r < warmup; ++r) {
      advance();
      pred->Run();
    }
    double ms = 0.0;
    for (int r = 0; r < repeat; ++r) {
      advance();
      const auto t0 = std::chrono::steady_clock::now();
      pred->Run();
      ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    const auto outs = pred->GetOutputNames();
    for (size_t i = 0; i < outs.size(); ++i) {
      auto h = pred->GetOutputHandle(outs[i]);
      const auto shp = h->shape();
      size_t n = 1;
      for (int d : shp) n *= (size_t)d;
      std::string dt;
      std::string bytes;
      switch (h->type()) {
        case DataType::FLOAT32:
        case DataType::FLOAT16:  // 16-bit outputs are written as float32
        case DataType::BFLOAT16:
          dt = "float32"; bytes.resize(n * 4); h->CopyToCpu(reinterpret_cast<float*>(&bytes[0])); break;
        case DataType::INT64: dt = "int64"; bytes.resize(n * 8); h->CopyToCpu(reinterpret_cast<int64_t*>(&bytes[0])); break;
        case DataType::INT32: dt = "int32"; bytes.resize(n * 4); h->CopyToCpu(reinterpret_cast<int32_t*>(&bytes[0])); break;
        default: throw std::runtime_error("unsupported output dtype");
      }
      std::ofstream f(outdir + "/" + std::to_string(i) + ".bin", std::ios::binary);
      f.write(bytes.data(), (std::streamsize)bytes.size());
      std::cout << "output " << i << " " << outs[i] << " " << dt << " ";
      for (size_t k = 0; k < shp.size(); ++k) std::cout << (k ? "," : "") << shp[k];
      std::cout << "\n";
    }
    std::cout << "run_ms " << ms / repeat << "\n" << GetVersion() << std::endl;
    pred.reset();  // tear the predictor down while the runtime is alive (and report it)
    std::cout << "released" << std::endl;
    return 0;
  } catch (const std::exception& e) {
    std::cerr << "error: " << e.what() << "\n";
    return 1;
  }
}
