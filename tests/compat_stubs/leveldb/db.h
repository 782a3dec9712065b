// Declaration stub for tests/test_app_compile.py only (syntax check of the reference's apps against include/).
#pragma once
#include <cstddef>
#include <string>
namespace leveldb {
class Slice {
 public:
  Slice(const char *d, size_t n);
  const char *data() const;
  size_t size() const;
};
class Status {
 public:
  bool ok() const;
  std::string ToString() const;
};
struct Options {
  bool create_if_missing = false;
  bool error_if_exists = false;
  size_t block_size = 4096;
  size_t write_buffer_size = 4 << 20;
};
struct ReadOptions {
  bool fill_cache = true;
};
struct WriteOptions {
  bool sync = false;
};
class Iterator {
 public:
  virtual ~Iterator();
  void SeekToFirst();
  bool Valid() const;
  void Next();
  Slice key() const;
  Slice value() const;
  Status status() const;
};
class DB {
 public:
  virtual ~DB();
  static Status Open(const Options &options, const std::string &name, DB **dbptr);
  Status Put(const WriteOptions &o, const Slice &key, const Slice &value);
  Iterator *NewIterator(const ReadOptions &o);
};
}  // namespace leveldb
