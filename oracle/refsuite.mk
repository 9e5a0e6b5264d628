# Build recipe for the REFERENCE's own known-answer test suites (test
# infrastructure only), compiled in place from the read-only reference tree:
#
#   tests/test-rules.c  (all rule groups, 3 iterator passes, test-rules.c:3694-3825)
#   tests/test-async.c  (interleaved scanners, ERROR_BLOCK_NOT_READY, :45-216)
#   tests/test-api.c    (scanner API, too-many-matches, flags, :43-996)
#   tests/util.c        (matches_blob / capture_string / test iterators)
#
# Two builds of each suite, into oracle/_ref/suite/:
#   <suite>       linked with the stock libyara (oracle/_ref/libyara_ref.so):
#                 the suites as upstream runs them (CPU, pins the fixtures)
#   <suite>-gpu   the same sources with every scan entry point renamed at
#                 compile time (REDIRECT) into integration/refsuite_gpu.c, which
#                 scans through the GPU integration (integration/_build/
#                 libyara_gpu_shim.so -> yara_amd/libyara_amd.so)
#
#   make -f oracle/refsuite.mk REF=/root/reference
#
# Needs oracle/ref.mk and integration/Makefile built first (__graft_entry__
# build() runs them in that order).  -DUSE_NO_PROC as SURVEY.md §8c: the
# process-scan test needs the tests/mapper helper, which cannot be built into
# the read-only tree.

REF ?= /root/reference
MAKEFLAGS += -r
.SUFFIXES:

OUT := oracle/_ref/suite
CC ?= gcc
CFLAGS_T := -O1 -g -D_GNU_SOURCE -DUSE_NO_PROC -DBUCKETS_128=1 -DCHECKSUM_1B=1 -w \
            -I$(REF)/libyara/include -I$(REF)/libyara -I$(REF)/tests

# every libyara entry point a suite scans through, and the destroy calls that
# end a YR_RULES / YR_SCANNER's lifetime (so the GPU twins are freed with them)
REDIRECT := -Dyr_rules_scan_mem=ygt_rules_scan_mem \
            -Dyr_rules_scan_mem_blocks=ygt_rules_scan_mem_blocks \
            -Dyr_rules_scan_file=ygt_rules_scan_file \
            -Dyr_rules_scan_fd=ygt_rules_scan_fd \
            -Dyr_rules_scan_proc=ygt_rules_scan_proc \
            -Dyr_rules_destroy=ygt_rules_destroy \
            -Dyr_scanner_scan_mem=ygt_scanner_scan_mem \
            -Dyr_scanner_scan_mem_blocks=ygt_scanner_scan_mem_blocks \
            -Dyr_scanner_scan_file=ygt_scanner_scan_file \
            -Dyr_scanner_scan_fd=ygt_scanner_scan_fd \
            -Dyr_scanner_scan_proc=ygt_scanner_scan_proc \
            -Dyr_scanner_destroy=ygt_scanner_destroy

REFLIB := -Loracle/_ref -lyara_ref -Wl,-rpath,'$$ORIGIN/..'
GPULIB := -Lintegration/_build -lyara_gpu_shim -Loracle/_ref -lyara_ref -Lyara_amd -lyara_amd \
          -Wl,-rpath,'$$ORIGIN/../../../integration/_build' -Wl,-rpath,'$$ORIGIN/..' \
          -Wl,-rpath,'$$ORIGIN/../../../yara_amd'

SUITES := test-rules test-async test-api

all: $(patsubst %,$(OUT)/%,$(SUITES)) $(patsubst %,$(OUT)/%-gpu,$(SUITES))

$(OUT):
	mkdir -p $(OUT)

$(OUT)/%: $(REF)/tests/%.c $(REF)/tests/util.c oracle/_ref/libyara_ref.so | $(OUT)
	$(CC) $(CFLAGS_T) $(REF)/tests/$*.c $(REF)/tests/util.c -o $@ $(REFLIB) -lpthread -lm

$(OUT)/refsuite_gpu.o: integration/refsuite_gpu.c integration/yr_gpu_scanner.h | $(OUT)
	$(CC) -O2 -D_GNU_SOURCE -Wall -I$(REF)/libyara/include -I$(REF)/libyara -c $< -o $@

$(OUT)/%-gpu: $(REF)/tests/%.c $(REF)/tests/util.c $(OUT)/refsuite_gpu.o \
              integration/_build/libyara_gpu_shim.so | $(OUT)
	$(CC) $(CFLAGS_T) $(REDIRECT) $(REF)/tests/$*.c $(REF)/tests/util.c $(OUT)/refsuite_gpu.o \
	  -o $@ $(GPULIB) -lpthread -lm

clean:
	rm -rf $(OUT)
.PHONY: all clean
