// Native HDF5 container writer (no libhdf5 on the target image).
//
// Reference: src/hdf5Lattice.cpp:26-339 writes one HDF5 file per output with one dataset per
// node-type group (uint8) and per quantity (float/double; vectors as [nz][ny][nx][3]) over
// the whole output region, every rank writing its hyperslab through parallel HDF5
// (H5Pset_fapl_mpio), chunked (chunk dims negotiated as the GCD of the ranks' local
// extents, src/Handlers/cbHDF5.cpp:98-126) and deflated at level 6 by default
// (cbHDF5.cpp:20-24, hdf5Lattice.cpp:125-134), plus an XDMF index.
//
// Here the file is laid out by hand in the classic ("HDF5 1.6") format, which every HDF5
// reader accepts:
//   superblock v0 | root group: object header v1 + symbol-table message -> v1 B-tree (one
//   leaf) + symbol-table node + local heap of names | one object header v1 per dataset
//   (dataspace v1, datatype v1, fill value v2, [filter pipeline v1: deflate], layout v3
//   contiguous or chunked) | chunk indexes (v1 B-trees of raw-data chunks, K = 32) | the
//   data blocks or chunks.
// No collective I/O library: every rank compresses its own chunks (tclb_h5_chunk_pack,
// OpenMP over chunks; a chunk never spans two ranks), rank 0 gathers the chunk sizes,
// writes the metadata and the chunk index and hands out the addresses
// (tclb_h5_create_chunked), then each rank writes its chunks at them (solver.py
// write_xdmf).  The contiguous form (tclb_h5_create) has its offsets known up front.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <sys/types.h>
#include <zlib.h>

#include <algorithm>
#include <array>
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

// one dataset of the file: contiguous (its data block placed after the metadata) or
// chunked (a v1 B-tree of raw-data chunks, optionally deflated, chunk addresses given)
struct Dataset {
  std::string name;
  int dtype = 0, rank = 0;
  uint64_t dims[4] = {0, 0, 0, 0};
  bool chunked = false;
  uint32_t cdims[4] = {0, 0, 0, 0};
  int level = -1;                      // deflate level, < 0: no filter
  // chunks: element offsets [rank] (global), stored size, file address (in/out)
  std::vector<std::array<uint64_t, 4>> coff;
  std::vector<uint64_t> csize, caddr;
  uint64_t addr = 0;                   // contiguous: the data block's address (out)
};

int esize(int dtype) { return dtype == 0 ? 1 : (dtype == 1 ? 4 : 8); }

constexpr int CHUNK_K = 32;   // indexed-storage B-tree K (superblock v0: the library default)

// the chunk index of a dataset: v1 B-tree (node type 1), leaves of up to 2K chunks,
// internal levels above; keys: chunk size, filter mask, element offsets (rank + 1, the
// last one 0); the final key of a node bounds its last chunk from above.  Returns the
// root address.
uint64_t chunk_btree(Buf& f, const Dataset& d) {
  const int nd = d.rank + 1;
  const size_t key = 8 + 8 * (size_t)nd;
  const size_t node_bytes = 24 + (2 * CHUNK_K + 1) * key + 2 * CHUNK_K * 8;
  std::vector<size_t> order(d.coff.size());
  for (size_t i = 0; i < order.size(); i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](size_t a, size_t b) {
    return std::lexicographical_compare(d.coff[a].begin(), d.coff[a].begin() + d.rank, d.coff[b].begin(),
                                        d.coff[b].begin() + d.rank);
  });
  // an entry of a level: its left key (chunk offsets), its size (leaf), address
  struct Ent {
    std::array<uint64_t, 4> off;
    uint64_t size, addr;
  };
  std::vector<Ent> cur;
  for (size_t i : order) cur.push_back({d.coff[i], d.csize[i], d.caddr[i]});
  std::array<uint64_t, 4> upper = cur.empty() ? std::array<uint64_t, 4>{0, 0, 0, 0} : cur.back().off;
  for (int k = 0; k < d.rank; k++) upper[k] += d.cdims[k];
  int level = 0;
  for (;;) {
    const size_t nn = (cur.size() + 2 * CHUNK_K - 1) / (2 * CHUNK_K);
    std::vector<Ent> up;
    std::vector<size_t> at(nn);
    for (size_t j = 0; j < nn; j++) {
      f.pad8();
      at[j] = f.pos();
      f.zeros(node_bytes);
    }
    for (size_t j = 0; j < nn; j++) {
      const size_t b0 = j * 2 * CHUNK_K, b1 = std::min(cur.size(), b0 + 2 * CHUNK_K);
      size_t p = at[j];
      memcpy(&f.b[p], "TREE", 4);
      f.b[p + 4] = 1;
      f.b[p + 5] = (uint8_t)level;
      f.b[p + 6] = (uint8_t)((b1 - b0) & 0xff);
      f.b[p + 7] = (uint8_t)((b1 - b0) >> 8);
      f.put64(p + 8, j > 0 ? at[j - 1] : UNDEF);
      f.put64(p + 16, j + 1 < nn ? at[j + 1] : UNDEF);
      p += 24;
      for (size_t e = b0; e <= b1; e++) {
        const bool last = e == b1;
        const std::array<uint64_t, 4>& o = last ? (b1 < cur.size() ? cur[b1].off : upper) : cur[e].off;
        f.put32(p, last || level > 0 ? 0 : cur[e].size);
        f.put32(p + 4, 0);                                   // filter mask: every filter applied
        for (int k = 0; k < nd; k++) f.put64(p + 8 + 8 * (size_t)k, k < d.rank ? o[k] : 0);
        p += key;
        if (!last) {
          f.put64(p, cur[e].addr);
          p += 8;
        }
      }
      up.push_back({cur[b0].off, 0, at[j]});
    }
    if (nn <= 1) return nn ? at[0] : UNDEF;
    cur.swap(up);
    level++;
  }
}

// the whole file: superblock, root group, dataset headers (and chunk B-trees), with the
// contiguous data blocks and the chunks placed after the metadata (64-byte aligned) in
// the given order.  Returns the file image of the metadata and its end-of-file address.
uint64_t layout_file(Buf& f, std::vector<Dataset>& ds) {
  const int n = (int)ds.size();
  std::vector<int> order(n);
  for (int i = 0; i < n; i++) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return ds[a].name < ds[b].name; });
  const int leafK = std::max(4, (n + 1) / 2 + 1);        // one symbol-table node holds all names
  const int internalK = 16;
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
    heapdata.bytes(ds[i].name.c_str(), ds[i].name.size() + 1);
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
    const Dataset& d = ds[i];
    uint64_t cnt = 1;
    for (int k = 0; k < d.rank; k++) cnt *= d.dims[k];
    nbytes[i] = cnt * esize(d.dtype);
    Buf sp;
    sp.u8(1); sp.u8(d.rank); sp.u8(0); sp.u8(0); sp.u32(0);
    for (int k = 0; k < d.rank; k++) sp.u64(d.dims[k]);
    Buf dt;
    datatype_msg(dt, d.dtype);
    Buf fv;
    // v2: allocation time early (contiguous) / incremental (chunked), never fill, undefined
    fv.u8(2); fv.u8(d.chunked ? 2 : 1); fv.u8(1); fv.u8(0);
    Buf lay;
    std::vector<std::pair<int, Buf>> msgs = {{0x1, sp}, {0x3, dt}, {0x5, fv}};
    if (d.chunked && d.level >= 0) {
      Buf pl;                                            // filter pipeline v1: deflate(level)
      pl.u8(1); pl.u8(1); pl.zeros(6);
      pl.u16(1); pl.u16(0); pl.u16(0); pl.u16(1);        // id 1, no name, mandatory, 1 value
      pl.u32((uint32_t)d.level);
      pl.u32(0);                                         // odd number of values: pad
      msgs.push_back({0xB, pl});
    }
    if (d.chunked) {
      lay.u8(3); lay.u8(2); lay.u8(d.rank + 1);          // v3, chunked, dimensionality
      lay.u64(0);                                        // B-tree address (patched)
      for (int k = 0; k < d.rank; k++) lay.u32(d.cdims[k]);
      lay.u32(esize(d.dtype));
    } else {
      lay.u8(3); lay.u8(1);                              // v3, contiguous
      lay.u64(0);                                        // data address (patched)
      lay.u64(nbytes[i]);
    }
    msgs.push_back({0x8, lay});
    f.pad8();
    oh[i] = f.pos();
    object_header(f, msgs);
    // address field of the layout message: last message, after its 8-byte header
    const size_t lay_body = f.pos() - ((lay.b.size() + 7) / 8) * 8;
    layout_addr[i] = lay_body + (d.chunked ? 3 : 2);
  }
  // ---- chunk B-trees: the chunk addresses are known once the metadata size is; the
  // B-tree size depends only on the chunk count, so size them first with dummy addresses
  size_t meta_end = f.pos();
  {
    Buf probe = f;
    for (int i = 0; i < n; i++)
      if (ds[i].chunked) {
        ds[i].caddr.assign(ds[i].coff.size(), 0);
        chunk_btree(probe, ds[i]);
      }
    probe.pad8();
    meta_end = probe.pos();
  }
  // ---- data placement (64-byte aligned): contiguous blocks, then chunks in given order
  uint64_t at = (meta_end + 63) / 64 * 64;
  std::vector<uint64_t> data_at(n, 0);
  for (int i = 0; i < n; i++) {
    Dataset& d = ds[i];
    if (!d.chunked) {
      data_at[i] = d.addr = at;
      at = (at + nbytes[i] + 63) / 64 * 64;
    } else {
      for (size_t c = 0; c < d.coff.size(); c++) {
        d.caddr[c] = at;
        at += d.csize[c];
      }
      at = (at + 63) / 64 * 64;
    }
  }
  for (int i = 0; i < n; i++) f.put64(layout_addr[i], ds[i].chunked ? chunk_btree(f, ds[i]) : data_at[i]);
  f.pad8();
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
  return at;
}

long long write_meta(const char* path, const Buf& f, uint64_t at) {
  FILE* fp = fopen(path, "wb");
  if (!fp) return -1;
  if (fwrite(f.b.data(), 1, f.pos(), fp) != f.pos()) { fclose(fp); return -1; }
  // size the file for the data (each rank writes its own blocks / chunks later)
  if (at > f.pos()) {
    if (fseeko(fp, (off_t)(at - 1), SEEK_SET) != 0 || fputc(0, fp) == EOF) { fclose(fp); return -1; }
  }
  fclose(fp);
  return (long long)at;
}

std::vector<Dataset> read_descs(int n, const char* names, const int* dtype, const int* rank,
                                const long long* dims) {
  std::vector<Dataset> ds(n);
  const char* p = names;
  for (int i = 0; i < n; i++) {
    ds[i].name = p;
    p += ds[i].name.size() + 1;
    ds[i].dtype = dtype[i];
    ds[i].rank = rank[i];
    for (int k = 0; k < rank[i]; k++) ds[i].dims[k] = (uint64_t)dims[4 * i + k];
  }
  return ds;
}

}  // namespace

extern "C" {

// Write the metadata of an HDF5 file holding n contiguous datasets and size it for their
// data.  names: n NUL-separated names; dtype[n] (0 uint8, 1 float32, 2 float64); rank[n]
// (1..4); dims[n*4] (slowest first).  offsets[n] receives the file offset of each data
// block.  Returns the file size, or -1 on an I/O error.
long long tclb_h5_create(const char* path, int n, const char* names, const int* dtype, const int* rank,
                         const long long* dims, long long* offsets) {
  std::vector<Dataset> ds = read_descs(n, names, dtype, rank, dims);
  Buf f;
  const uint64_t at = layout_file(f, ds);
  for (int i = 0; i < n; i++) offsets[i] = (long long)ds[i].addr;
  return write_meta(path, f, at);
}

// Chunked datasets (reference hdf5WriteLattice: H5Pset_chunk + H5Pset_deflate(6)).
// cdims[n*4]: chunk dims; level: deflate level (< 0: no filter); nchunks[n]: chunks per
// dataset; coff[sum nchunks * 4]: their element offsets; csize[sum nchunks]: stored bytes.
// The chunks of a dataset are placed in the order given (callers list each rank's chunks
// consecutively, so a rank writes one run); caddr[sum nchunks] receives the addresses.
long long tclb_h5_create_chunked(const char* path, int n, const char* names, const int* dtype, const int* rank,
                                 const long long* dims, const long long* cdims, int level, const long long* nchunks,
                                 const long long* coff, const long long* csize, long long* caddr) {
  std::vector<Dataset> ds = read_descs(n, names, dtype, rank, dims);
  long long c0 = 0;
  for (int i = 0; i < n; i++) {
    Dataset& d = ds[i];
    d.chunked = true;
    d.level = level;
    for (int k = 0; k < d.rank; k++) d.cdims[k] = (uint32_t)cdims[4 * i + k];
    for (long long c = 0; c < nchunks[i]; c++) {
      std::array<uint64_t, 4> o = {0, 0, 0, 0};
      for (int k = 0; k < d.rank; k++) o[k] = (uint64_t)coff[4 * (c0 + c) + k];
      d.coff.push_back(o);
      d.csize.push_back((uint64_t)csize[c0 + c]);
    }
    c0 += nchunks[i];
  }
  Buf f;
  const uint64_t at = layout_file(f, ds);
  c0 = 0;
  for (int i = 0; i < n; i++)
    for (size_t c = 0; c < ds[i].caddr.size(); c++) caddr[c0++] = (long long)ds[i].caddr[c];
  return write_meta(path, f, at);
}

// Compress the chunks of one rank's local block: data [d0][d1]...[d_{rank-1}] (element
// size es), chunk dims cd (dividing every local dim), chunk order row-major over the chunk
// grid.  level >= 0: zlib deflate (the HDF5 deflate filter's format), else raw copies.
// out: room for tclb_h5_chunk_bound() bytes; sizes[nchunks] receives each chunk's size.
// Chunks are compressed in parallel (OpenMP).  Returns the total size, -1 on an error.
long long tclb_h5_chunk_bound(int es, int rank, const long long* ld, const long long* cd) {
  long long nch = 1, ce = 1;
  for (int k = 0; k < rank; k++) {
    nch *= ld[k] / cd[k];
    ce *= cd[k];
  }
  return nch * (long long)compressBound((uLong)(ce * es));
}

long long tclb_h5_chunk_pack(const void* data, int es, int rank, const long long* ld, const long long* cd, int level,
                             void* out, long long* sizes) {
  long long ng[4] = {1, 1, 1, 1}, ce = 1, nch = 1;
  for (int k = 0; k < rank; k++) {
    if (cd[k] <= 0 || ld[k] % cd[k] != 0) return -1;
    ng[k] = ld[k] / cd[k];
    ce *= cd[k];
    nch *= ng[k];
  }
  const long long cbytes = ce * es;
  const long long bound = (long long)compressBound((uLong)cbytes);
  int err = 0;
#pragma omp parallel
  {
    std::vector<uint8_t> tmp((size_t)cbytes);
#pragma omp for schedule(dynamic)
    for (long long c = 0; c < nch; c++) {
      // gather chunk c (row-major over the chunk grid) into tmp
      long long idx[4] = {0, 0, 0, 0}, r = c;
      for (int k = rank - 1; k >= 0; k--) {
        idx[k] = r % ng[k];
        r /= ng[k];
      }
      const long long row = cd[rank - 1] * es;
      const long long nrows = ce / cd[rank - 1];
      for (long long q = 0; q < nrows; q++) {
        long long rem = q, src = 0, stride = 1;
        long long pos[4] = {0, 0, 0, 0};
        for (int k = rank - 2; k >= 0; k--) {
          pos[k] = rem % cd[k];
          rem /= cd[k];
        }
        for (int k = rank - 1; k >= 0; k--) {
          const long long g = idx[k] * cd[k] + (k == rank - 1 ? 0 : pos[k]);
          src += g * stride;
          stride *= ld[k];
        }
        memcpy(&tmp[(size_t)(q * row)], (const uint8_t*)data + src * es, (size_t)row);
      }
      uint8_t* dst = (uint8_t*)out + c * bound;
      if (level >= 0) {
        uLongf n = (uLongf)bound;
        if (compress2(dst, &n, tmp.data(), (uLong)cbytes, level) != Z_OK) {
#pragma omp atomic write
          err = 1;
        }
        sizes[c] = (long long)n;
      } else {
        memcpy(dst, tmp.data(), (size_t)cbytes);
        sizes[c] = cbytes;
      }
    }
  }
  if (err) return -1;
  // close the gaps: chunk c moves from c * bound to the running offset
  long long at = 0;
  for (long long c = 0; c < nch; c++) {
    if (at != c * bound) memmove((uint8_t*)out + at, (uint8_t*)out + c * bound, (size_t)sizes[c]);
    at += sizes[c];
  }
  return at;
}

}  // extern "C"
