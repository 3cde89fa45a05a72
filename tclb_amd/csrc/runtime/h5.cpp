// Native HDF5 container writer (no libhdf5 on the target image).
//
// Reference: src/hdf5Lattice.cpp:26-339 writes one HDF5 file per output with one dataset per
// node-type group (uint8) and per quantity (float/double; vectors as [nz][ny][nx][3]) over
// the whole output region, every rank writing its hyperslab through parallel HDF5
// (H5Pset_fapl_mpio), plus an XDMF index.
//
// Here the file is laid out by hand in the classic ("HDF5 1.6") format, which every HDF5
// reader accepts:
//   superblock v0 | root group: object header v1 + symbol-table message -> v1 B-tree (one
//   leaf) + symbol-table node + local heap of names | one object header v1 per dataset
//   (dataspace v1, datatype v1, fill value v2, contiguous layout v3) | the raw data blocks.
// Datasets are contiguous and their file offsets are known when the file is created, so
// every rank writes its own hyperslab straight into the file (pwrite / memory map) with no
// collective I/O library: tclb_h5_create() writes the metadata (rank 0), then each rank
// fills its part of the data blocks (tclb_amd/io/hdf5.py).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

namespace {

const uint64_t UNDEF = ~0ull;

struct Buf {
  std::vector<uint8_t> b;
  size_t pos() const { return b.size(); }
  void u8(uint64_t v) { b.push_back((uint8_t)v); }
  void u16(uint64_t v) { for (int i = 0; i < 2; i++) u8(v >> (8 * i)); }
  void u32(uint64_t v) { for (int i = 0; i < 4; i++) u8(v >> (8 * i)); }
  void u64(uint64_t v) { for (int i = 0; i < 8; i++) u8(v >> (8 * i)); }
  void bytes(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  void pad8() { while (b.size() % 8) u8(0); }
  void zeros(size_t n) { b.insert(b.end(), n, 0); }
  void put64(size_t at, uint64_t v) { for (int i = 0; i < 8; i++) b[at + i] = (uint8_t)(v >> (8 * i)); }
  void put32(size_t at, uint64_t v) { for (int i = 0; i < 4; i++) b[at + i] = (uint8_t)(v >> (8 * i)); }
};

// datatype message (class, size, properties): dtype 0 = uint8, 1 = float32, 2 = float64
void datatype_msg(Buf& m, int dtype) {
  if (dtype == 0) {
    m.u8(0x10);                 // version 1, class 0 (fixed point)
    m.u8(0x00); m.u8(0); m.u8(0);   // little endian, unsigned
    m.u32(1);
    m.u16(0); m.u16(8);         // bit offset, precision
  } else {
    const bool d = dtype == 2;
    m.u8(0x11);                 // version 1, class 1 (floating point)
    m.u8(0x20);                 // little endian, implied-msb mantissa normalisation
    m.u8(d ? 63 : 31);          // sign bit location
    m.u8(0);
    m.u32(d ? 8 : 4);
    m.u16(0); m.u16(d ? 64 : 32);               // bit offset, precision
    m.u8(d ? 52 : 23); m.u8(d ? 11 : 8);        // exponent location, size
    m.u8(0); m.u8(d ? 52 : 23);                 // mantissa location, size
    m.u32(d ? 1023 : 127);                      // exponent bias
  }
}

// one header message: type, size (padded to 8), flags, body
void message(Buf& h, int type, const Buf& body, int flags = 0) {
  Buf p = body;
  p.pad8();
  h.u16(type);
  h.u16(p.b.size());
  h.u8(flags);
  h.zeros(3);
  h.bytes(p.b.data(), p.b.size());
}

// object header v1 holding the given messages
void object_header(Buf& f, const std::vector<std::pair<int, Buf>>& msgs) {
  Buf body;
  for (auto& m : msgs) message(body, m.first, m.second, m.first == 3 ? 1 : 0);   // datatype: constant
  f.u8(1); f.u8(0);             // version 1, reserved
  f.u16(msgs.size());
  f.u32(1);                     // reference count
  f.u32(body.b.size());
  f.zeros(4);                   // pad the 12-byte prefix to 16
  f.bytes(body.b.data(), body.b.size());
}

}  // namespace

extern "C" {

// Write the metadata of an HDF5 file holding n contiguous datasets and size it for their
// data.  names: n NUL-separated names; dtype[n] (0 uint8, 1 float32, 2 float64); rank[n]
// (1..4); dims[n*4] (slowest first).  offsets[n] receives the file offset of each data
// block.  Returns the file size, or -1 on an I/O error.
long long tclb_h5_create(const char* path, int n, const char* names, const int* dtype, const int* rank,
                         const long long* dims, long long* offsets) {
  std::vector<std::string> nm;
  const char* p = names;
  for (int i = 0; i < n; i++) {
    nm.emplace_back(p);
    p += nm.back().size() + 1;
  }
  // symbol-table entries must be sorted by name (the B-tree key order)
  std::vector<int> order(n);
  for (int i = 0; i < n; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return nm[a] < nm[b]; });
  const int leafK = std::max(4, (n + 1) / 2 + 1);        // one symbol-table node holds all names
  const int internalK = 16;

  Buf f;
  // ---- superblock v0 (96 bytes)
  const unsigned char sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
  f.bytes(sig, 8);
  f.u8(0); f.u8(0); f.u8(0); f.u8(0); f.u8(0);
  f.u8(8); f.u8(8); f.u8(0);    // size of offsets, lengths
  f.u16(leafK); f.u16(internalK);
  f.u32(0);                     // file consistency flags
  f.u64(0);                     // base address
  f.u64(UNDEF);                 // free-space info
  const size_t eof_at = f.pos();
  f.u64(0);                     // end of file (patched)
  f.u64(UNDEF);                 // driver info
  // root group symbol-table entry
  f.u64(0);                     // link name offset
  const size_t root_oh_at = f.pos();
  f.u64(0);                     // object header address (patched)
  f.u32(1); f.u32(0);           // cache type 1: B-tree + heap in the scratch pad
  const size_t root_scratch = f.pos();
  f.u64(0); f.u64(0);
  f.pad8();

  // ---- local heap of names: "" at offset 0, then every name (8-byte aligned)
  Buf heapdata;
  heapdata.zeros(8);
  std::vector<uint64_t> name_off(n);
  for (int i = 0; i < n; i++) {
    name_off[i] = heapdata.pos();
    heapdata.bytes(nm[i].c_str(), nm[i].size() + 1);
    heapdata.pad8();
  }
  // ---- root object header: symbol-table message (B-tree, heap addresses patched)
  f.pad8();
  const size_t root_oh = f.pos();
  {
    Buf stm;
    stm.u64(0); stm.u64(0);
    object_header(f, {{0x11, stm}});
  }
  const size_t stm_at = root_oh + 16 + 8;     // the message body after prefix + message header
  f.pad8();
  // local heap header
  const size_t heap_at = f.pos();
  f.bytes("HEAP", 4); f.u8(0); f.zeros(3);
  f.u64(heapdata.pos());        // data segment size
  f.u64(1);                     // free-list head: none (libhdf5's H5HL_FREE_NULL = 1)
  const size_t heap_data_ptr = f.pos();
  f.u64(0);
  f.pad8();
  const size_t heap_data_at = f.pos();
  f.bytes(heapdata.b.data(), heapdata.pos());
  f.pad8();
  f.put64(heap_data_ptr, heap_data_at);
  // B-tree v1, group node, one leaf entry -> the symbol-table node
  const size_t btree_at = f.pos();
  f.bytes("TREE", 4);
  f.u8(0); f.u8(0);             // node type 0 (group), level 0
  f.u16(n > 0 ? 1 : 0);         // entries used
  f.u64(UNDEF); f.u64(UNDEF);   // siblings
  const size_t btree_keys = f.pos();
  // room for 2K children: keys (2K+1) x 8 + children 2K x 8
  f.zeros((2 * internalK + 1) * 8 + 2 * internalK * 8);
  f.pad8();
  // symbol-table node
  const size_t snod_at = f.pos();
  f.bytes("SNOD", 4);
  f.u8(1); f.u8(0);
  f.u16(n);
  const size_t entries_at = f.pos();
  f.zeros((size_t)2 * leafK * 40);
  f.pad8();
  if (n > 0) {
    f.put64(btree_keys, 0);                              // key 0: "" (heap offset 0)
    f.put64(btree_keys + 8, snod_at);                    // child 0
    f.put64(btree_keys + 16, name_off[order[n - 1]]);    // key 1: largest name
  }
  // ---- dataset object headers
  std::vector<size_t> oh(n), layout_addr(n);
  std::vector<uint64_t> nbytes(n);
  for (int i = 0; i < n; i++) {
    uint64_t cnt = 1;
    for (int k = 0; k < rank[i]; k++) cnt *= (uint64_t)dims[4 * i + k];
    nbytes[i] = cnt * (dtype[i] == 0 ? 1 : (dtype[i] == 1 ? 4 : 8));
    Buf ds;
    ds.u8(1); ds.u8(rank[i]); ds.u8(0); ds.u8(0); ds.u32(0);
    for (int k = 0; k < rank[i]; k++) ds.u64(dims[4 * i + k]);
    Buf dt;
    datatype_msg(dt, dtype[i]);
    Buf fv;
    fv.u8(2); fv.u8(1); fv.u8(1); fv.u8(0);            // v2: early allocation, never fill, undefined
    Buf lay;
    lay.u8(3); lay.u8(1);                              // v3, contiguous
    lay.u64(0);                                        // data address (patched)
    lay.u64(nbytes[i]);
    f.pad8();
    oh[i] = f.pos();
    object_header(f, {{0x1, ds}, {0x3, dt}, {0x5, fv}, {0x8, lay}});
    // address field of the layout message: last message, after its 8-byte header and 2 bytes
    const size_t lay_body = f.pos() - ((lay.b.size() + 7) / 8) * 8;
    layout_addr[i] = lay_body + 2;
  }
  f.pad8();
  // ---- data blocks (64-byte aligned)
  uint64_t at = (f.pos() + 63) / 64 * 64;
  for (int i = 0; i < n; i++) {
    offsets[i] = (long long)at;
    f.put64(layout_addr[i], at);
    at = (at + nbytes[i] + 63) / 64 * 64;
  }
  // ---- patch the root entry and the symbol-table node entries
  f.put64(eof_at, at);
  f.put64(root_oh_at, root_oh);
  f.put64(root_scratch, btree_at);
  f.put64(root_scratch + 8, heap_at);
  f.put64(stm_at, btree_at);
  f.put64(stm_at + 8, heap_at);
  for (int j = 0; j < n; j++) {
    const int i = order[j];
    const size_t e = entries_at + (size_t)j * 40;
    f.put64(e, name_off[i]);
    f.put64(e + 8, oh[i]);
    f.put32(e + 16, 0);         // cache type 0
  }
  FILE* fp = fopen(path, "wb");
  if (!fp) return -1;
  if (fwrite(f.b.data(), 1, f.pos(), fp) != f.pos()) { fclose(fp); return -1; }
  // size the file for the data blocks (each rank writes its hyperslabs later)
  if (at > f.pos()) {
    if (fseek(fp, (long)(at - 1), SEEK_SET) != 0 || fputc(0, fp) == EOF) { fclose(fp); return -1; }
  }
  fclose(fp);
  return (long long)at;
}

}  // extern "C"
