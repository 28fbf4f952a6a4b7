/*
 * pn2io.h -- C ABI of libpn2io.so: the dataset text reader that feeds the path (SURVEY.md
 * §8(f) rank 4), host code (C++17, no GPU).
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   pn2io_read_csv_f64   np.loadtxt(path, delimiter=",") of one point / _rot / _tran file
 *                                              data_utils/ModelDataLoader.py:85-90
 *   pn2io_read_many_f64  the same for a batch of files, parsed on a thread pool (the
 *                        DataLoader's per-item loadtxt calls, ModelDataLoader.py:78-91)
 * Files are the ones the data_build scripts write with np.savetxt(fmt='%6f', delimiter=",")
 * (data_build/Cube.py:90-94): one row per point, `cols` numbers per row.
 *
 * Parsing matches np.loadtxt(delimiter=...) bit for bit: each field is converted with a
 * correctly rounded decimal -> double conversion (std::from_chars; numpy uses
 * PyOS_string_to_double, also correctly rounded), surrounding blanks and a leading '+' are
 * accepted, text from '#' to the end of a line is a comment, blank lines are skipped, and a row
 * with another number of fields is an error (numpy raises ValueError).
 *
 * Return: 0, or a negative PN2IO_E* code with a thread-local message (pn2io_last_error).
 * No global mutable state: calls are re-entrant across threads.
 */
#ifndef PN2IO_H
#define PN2IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PN2IO_OK 0
#define PN2IO_EIO (-1)     /* cannot open / read the file */
#define PN2IO_EPARSE (-2)  /* a field is not a number, or a row has another field count */
#define PN2IO_ESIZE (-3)   /* more rows than the output holds */
#define PN2IO_EINVAL (-4)  /* bad argument */

#define PN2IO_ABI_VERSION 1
int pn2io_abi_version(void);
const char *pn2io_last_error(void);

/* Rows and columns of a delimited text file (cols of its first data row). */
int pn2io_shape(const char *path, char delim, int64_t *rows, int64_t *cols);

/* Parse `path` into out[max_rows][cols] (row-major float64); *rows_out = data rows read. */
int pn2io_read_csv_f64(const char *path, char delim, int64_t cols, int64_t max_rows,
                       double *out, int64_t *rows_out);

/* n files on up to `threads` threads (<= 0: hardware concurrency): file i into
 * out + i*max_rows*cols, its row count into rows_out[i].  The first failing file (lowest i)
 * sets the returned code and message; every file is attempted. */
int pn2io_read_many_f64(const char *const *paths, int64_t n, char delim, int64_t cols,
                        int64_t max_rows, double *out, int64_t *rows_out, int threads);

#ifdef __cplusplus
}
#endif
#endif /* PN2IO_H */
