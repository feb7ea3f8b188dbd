/*
 * dec_prelude.h -- TEST INFRASTRUCTURE: forced include (-include) of the
 * decoder build of the reference, oracle/_ref/libhl_dec.a (oracle/Makefile).
 *
 * The reference's one-bit reader (hl_codec_264_bits.h:201-217) has a GNU
 * inline-asm branch whose operand names do not assemble; its portable branch
 * is selected when __GNUC__ is not defined.  This prelude includes the system
 * headers and the reference's own hl_config.h while __GNUC__ is still
 * defined (so glibc and the reference's alignment / inline macros keep their
 * GNU definitions), then undefines __GNUC__ for the rest of the translation
 * unit.  Nothing of the reference is replaced or redefined.
 */
#include <limits.h>
#include <string.h>
#include <stdint.h>
#include <stddef.h>
#include <stdarg.h>
#include <stdio.h>
#include <ctype.h>
#include <stdlib.h>
#include <assert.h>
#include <pthread.h>
#include <time.h>
#include <sys/time.h>
#include <sys/stat.h>
#include <errno.h>
#include <math.h>
#include <unistd.h>
#include <semaphore.h>
#include <sched.h>
#include <malloc.h>
#include <fcntl.h>
#include <dlfcn.h>
#include <float.h>
#include <byteswap.h>
#include <hl_config.h>
#undef __GNUC__
