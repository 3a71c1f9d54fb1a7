// cdc_example.cpp -- the C++ host mirror in use (counterpart of the
// reference's examples/cdc.rs and of SURVEY.md §8d config 1).
//
//   g++ -std=c++17 -O2 -Iinclude examples/cdc_example.cpp -Lchunkfs_amd
//       -lchunkfs_amd -Wl,-rpath,'$ORIGIN/../chunkfs_amd' -o _build/cdc_example
//
// Writes a 64 MiB splitmix64 buffer through FSChunker(8 KiB) and through
// FastChunker(4/8/16 KiB) -- whole buffer and via the 1 MiB write path -- and
// prints chunk counts; exits non-zero if an invariant fails.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <numeric>

#include "chunkfs_amd.hpp"

using namespace chunkfs_amd;

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main() {
    const size_t n = 64 * MB;
    std::vector<uint8_t> data(n);
    for (size_t i = 0; i < n / 8; ++i) {
        const uint64_t w = mix64(0x0C0FFEE1ull + (i + 1) * 0x9E3779B97F4A7C15ull);
        std::memcpy(&data[8 * i], &w, 8);
    }
    try {
        FSChunker fs(8 * KB);
        const auto fixed = fs.chunk_data(data);
        std::printf("%s: %zu chunks\n", fs.debug().c_str(), fixed.size());
        if (fixed.size() != 8192) return 2;

        FastChunker fast(SizeParams{4 * KB, 8 * KB, 16 * KB});
        const auto t0 = std::chrono::steady_clock::now();
        const auto chunks = fast.chunk_data(data);
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        size_t total = 0;
        for (const auto &c : chunks) total += c.length();
        std::printf("%s: %zu chunks, avg %.0f B, %.2f GiB/s incl. H2D/D2H\n", fast.debug().c_str(),
                    chunks.size(), (double)n / chunks.size(), n / s / GB);
        if (total != n || chunks.front().offset() != 0) return 3;

        double chunk_s = 0;
        const auto spans = fast.write_spans(data.data(), n, &chunk_s);
        if (spans.size() != chunks.size()) return 4;
        for (size_t i = 0; i < spans.size(); ++i)
            if (spans[i] != chunks[i].length()) return 5;  // segmentation invariance
        std::printf("write path: %zu spans == whole-buffer chunks; chunk_data time %.3f s\n", spans.size(), chunk_s);

        // The other chunker families (segment-walk engine): tiling + the
        // same segmentation invariance through the write path.
        const SizeParams sz{4 * KB, 8 * KB, 16 * KB};
        std::vector<std::unique_ptr<Chunker>> others;
        others.emplace_back(new RabinChunker(sz));
        others.emplace_back(new UltraChunker(sz));
        others.emplace_back(new LeapChunker(sz));
        others.emplace_back(new SeqChunker(OperationMode::Increasing, sz));
        for (auto &ch : others) {
            const auto oc = ch->chunk_data(data);
            size_t tot = 0;
            for (const auto &c : oc) tot += c.length();
            if (tot != n || oc.front().offset() != 0) return 6;
            const auto os = ch->write_spans(data.data(), n);
            if (os.size() != oc.size()) return 7;
            for (size_t i = 0; i < os.size(); ++i)
                if (os[i] != oc[i].length()) return 8;
            std::printf("%s: %zu chunks, write path identical\n", ch->debug().c_str(), oc.size());
        }
    } catch (const Error &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
