// fc2_gzpieces.h -- spliced_reads.fastq.gz written by the native read loop: the text is cut into
// pieces, each compressed as its own gzip member on worker threads and written in order.
// Concatenated members are one valid gzip stream (RFC 1952 2.2), so every reader sees the same
// text as from one member (the Python writer, find_circ2_amd/gzout.py, does the same).  Used from
// one thread (the side that records chunks); the workers only compress.
#pragma once
#include <stdio.h>
#include <zlib.h>

#include "fc2_cpuacct.h"
#include "fc2_deflate.h"

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace fc2 {

class GzPieces {
  public:
    ~GzPieces() {
        std::string err;
        close(err);
    }
    bool is_open() const { return f_ != nullptr; }

    bool open(const char *path, int level, int threads, size_t piece, std::string &err) {
        f_ = fopen(path, "wb");
        if (!f_) { err = std::string("IOError: cannot open '") + path + "' for writing"; return false; }
        level_ = level;
        piece_ = piece ? piece : (size_t(4) << 20);
        const int n = threads > 0 ? threads : 1;
        max_pending_ = 2 * (size_t)n;
        stop_ = false;
        for (int k = 0; k < n; ++k) th_.emplace_back([this] { worker(); });
        return true;
    }

    // takes the bytes of text (text is left empty, its capacity kept for the caller's next chunk);
    // whole pieces go to the workers, each byte is copied once
    void append(std::string &text) {
        size_t at = 0;
        if (!buf_.empty()) {                    // top up the partial piece left by the last call
            at = std::min(piece_ - buf_.size(), text.size());
            buf_.append(text, 0, at);
            if (buf_.size() >= piece_) {
                submit(std::move(buf_));
                buf_.clear();
            }
        }
        while (text.size() - at >= piece_) {
            submit(text.substr(at, piece_));
            at += piece_;
        }
        buf_.append(text, at, std::string::npos);
        text.clear();
    }

    // takes `text` whole as the next member (after what append() left pending) if it is at most two
    // pieces long, leaving `text` empty with a recycled buffer's capacity: a chunk's range texts go
    // out without being copied
    void append_owned(std::string &text) {
        if (text.empty()) return;
        if (text.size() > 2 * piece_) {         // members stay about a piece long
            append(text);
            return;
        }
        if (!buf_.empty()) {
            submit(std::move(buf_));
            buf_.clear();
        }
        std::string fresh;
        {
            std::lock_guard<std::mutex> lk(m_);
            if (!spare_.empty()) {
                fresh.swap(spare_.back());
                spare_.pop_back();
            }
        }
        fresh.swap(text);                       // text: the recycled buffer, emptied
        text.clear();
        submit(std::move(fresh));
    }

    // compresses what is left, writes every member, stops the workers; false on a write error
    bool close(std::string &err) {
        if (!f_) return true;
        if (!buf_.empty() || !wrote_any_) submit(std::move(buf_));   // an empty file still gets one member
        buf_.clear();
        while (!order_.empty()) write_front();
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_work_.notify_all();
        for (std::thread &t : th_) t.join();
        th_.clear();
        const bool ok = !werr_ && fclose(f_) == 0;
        f_ = nullptr;
        if (!ok) err = "IOError: writing spliced_reads.fastq.gz failed";
        return ok;
    }

  private:
    struct Job {
        std::string in, out;
        bool done = false;
        bool zerr = false;
    };
    FILE *f_ = nullptr;
    int level_ = 6;
    size_t piece_ = size_t(4) << 20, max_pending_ = 2;
    std::string buf_;
    std::deque<std::shared_ptr<Job>> order_;   // submission order: written front first
    std::deque<std::shared_ptr<Job>> work_;    // not yet taken by a worker
    std::mutex m_;
    std::condition_variable cv_work_, cv_done_;
    std::vector<std::thread> th_;
    bool stop_ = false, werr_ = false, wrote_any_ = false;
    std::vector<std::string> spare_;           // compressed inputs' buffers, for append_owned

    void submit(std::string &&data) {
        auto j = std::make_shared<Job>();
        j->in = std::move(data);
        {
            std::lock_guard<std::mutex> lk(m_);
            work_.push_back(j);
        }
        cv_work_.notify_one();
        order_.push_back(j);
        wrote_any_ = true;
        while (order_.size() > max_pending_) write_front();
    }

    void write_front() {
        std::shared_ptr<Job> j = order_.front();
        {
            std::unique_lock<std::mutex> lk(m_);
            cv_done_.wait(lk, [&] { return j->done; });
        }
        order_.pop_front();
        if (j->zerr || (!j->out.empty() && fwrite(j->out.data(), 1, j->out.size(), f_) != j->out.size())) werr_ = true;
    }

    void worker() {
        for (;;) {
            std::shared_ptr<Job> j;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_work_.wait(lk, [&] { return stop_ || !work_.empty(); });
                if (work_.empty()) return;
                j = work_.front();
                work_.pop_front();
            }
            compress(*j);
            {
                std::lock_guard<std::mutex> lk(m_);
                j->done = true;
            }
            cv_done_.notify_all();
        }
    }

    void compress(Job &j) {
        cpu::Scope acct(cpu::GZIP);
        if (!dfl::gzip_member(j.in, level_, j.out)) j.zerr = true;   // libdeflate, or zlib (fc2_deflate.h)
        j.in.clear();
        std::lock_guard<std::mutex> lk(m_);
        if (spare_.size() < 2 * max_pending_) spare_.push_back(std::move(j.in));
        std::string().swap(j.in);
    }
};

}  // namespace fc2
