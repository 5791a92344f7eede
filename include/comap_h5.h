/* comap_h5.h -- native HDF5 I/O for the Level-1 / Level-2 wire format.
 *
 * Replaces the h5py calls of the reference's file layer (h5py is not in this
 * image; libhdf5 1.10 is, under /opt/conda):
 *   - HDF5Data.read_data_file / hdf5_visitor_function
 *       comancpipeline/Analysis/DataHandling.py:101-108, 168-179
 *     -> comap_h5_open(mode 0) + comap_h5_visit + comap_h5_info/read (+ attrs);
 *        large datasets (spectrometer/tod) stay lazy: comap_h5_read (hyperslab)
 *        and comap_h5_read_flat (a flat element range, the staging unit of the
 *        pinned host->device upload)
 *   - HDF5Data.write_data_file / create_groups  DataHandling.py:110-166
 *     -> comap_h5_open(mode 1) + comap_h5_write (intermediate groups created,
 *        an existing dataset replaced) + comap_h5_attr_write
 *   - the Level-2 readers of the map-maker, h5py.File(filename, 'r')
 *       comancpipeline/MapMaking/COMAPData.py:170, 252, 389, 435
 *
 * Types follow h5py's mapping so files interoperate both ways: numpy bool is
 * the int8 enum {FALSE, TRUE}; str is a variable-length UTF-8 string; bytes /
 * numpy 'S' are fixed-length NULLPAD strings.
 *
 * Conventions: int status (0 ok, < 0 error), comap_h5_last_error() (per
 * thread); the listing calls return the bytes they need (call again with a
 * larger buffer); one handle is not to be used from two threads at once.
 */
#ifndef COMAP_H5_H
#define COMAP_H5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct comap_h5 comap_h5;

enum comap_h5_dtype {
    COMAP_H5_F32 = 1, COMAP_H5_F64 = 2,
    COMAP_H5_I8 = 3, COMAP_H5_I16 = 4, COMAP_H5_I32 = 5, COMAP_H5_I64 = 6,
    COMAP_H5_U8 = 7, COMAP_H5_U16 = 8, COMAP_H5_U32 = 9, COMAP_H5_U64 = 10,
    COMAP_H5_BOOL = 11,
    COMAP_H5_STR_FIXED = 12,   /* elsize bytes per element, NUL padded */
    COMAP_H5_STR_VLEN = 13,    /* variable-length UTF-8 (comap_h5_*_strings) */
    COMAP_H5_UNSUPPORTED = 0
};

#define COMAP_H5_MAX_RANK 32

const char *comap_h5_version(void);
const char *comap_h5_last_error(void);

/* mode 0: read only; 1: read/write, created when missing ('a'); 2: truncate ('w') */
int comap_h5_open(const char *path, int32_t mode, comap_h5 **out);
int comap_h5_close(comap_h5 *f);
int comap_h5_flush(comap_h5 *f);

/* 1 when an object (group or dataset) exists at path, 0 when not */
int comap_h5_exists(comap_h5 *f, const char *path);
/* every object below the root, depth first in name order (h5py visititems):
 * lines "D <path>\n" (dataset) or "G <path>\n" (group); returns the bytes needed */
int64_t comap_h5_visit(comap_h5 *f, char *buf, int64_t cap);
int comap_h5_require_group(comap_h5 *f, const char *path);
int comap_h5_delete(comap_h5 *f, const char *path);

/* dataset type and shape: dims holds COMAP_H5_MAX_RANK entries */
int comap_h5_info(comap_h5 *f, const char *path, int32_t *dtype, int32_t *ndim, int64_t *dims, int64_t *elsize);
/* hyperslab [start, start + count) (NULL start/count: the whole dataset), row-major into buf */
int comap_h5_read(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, const int64_t *start,
                  const int64_t *count, void *buf);
/* elements [offset, offset + n) of the row-major flattened dataset */
int comap_h5_read_flat(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, int64_t offset, int64_t n,
                       void *buf);
/* creates intermediate groups and replaces an existing object at path */
int comap_h5_write(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, int32_t ndim, const int64_t *dims,
                   const void *buf);

/* variable-length strings of a dataset (attr == NULL) or of attribute attr of
 * the object at path: NUL-terminated, back to back; returns the bytes needed */
int64_t comap_h5_read_strings(comap_h5 *f, const char *path, const char *attr, char *buf, int64_t cap);
/* writes n = prod(dims) NUL-terminated strings from buf as variable-length UTF-8 */
int comap_h5_write_strings(comap_h5 *f, const char *path, const char *attr, int32_t ndim, const int64_t *dims,
                           const char *buf);

/* attribute names of the object at path, one per line; returns the bytes needed */
int64_t comap_h5_attr_list(comap_h5 *f, const char *path, char *buf, int64_t cap);
int comap_h5_attr_info(comap_h5 *f, const char *path, const char *name, int32_t *dtype, int32_t *ndim,
                       int64_t *dims, int64_t *elsize);
int comap_h5_attr_read(comap_h5 *f, const char *path, const char *name, int32_t dtype, int64_t elsize, void *buf);
/* replaces an existing attribute; the object at path must exist */
int comap_h5_attr_write(comap_h5 *f, const char *path, const char *name, int32_t dtype, int64_t elsize,
                        int32_t ndim, const int64_t *dims, const void *buf);

#ifdef __cplusplus
}
#endif

#endif /* COMAP_H5_H */
