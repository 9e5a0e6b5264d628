# Build recipe for the REFERENCE libyara 4.2.1 (test infrastructure only).
#
# Compiles the reference C sources in place (read-only, never copied) into
# oracle/_ref/.  Nothing here is product code: the artefacts are the oracle the
# parity tests and bench.py's cpu_baseline leg check the HIP path against.
#
#   make -f oracle/ref.mk REF=/root/reference -j8
#
# Outputs (git-ignored, but travel to the GPU box with the gpurun snapshot):
#   oracle/_ref/libyara_ref.so   stock libyara (scanner.c, scan.c, exec.c, ... as-is)
#   oracle/_ref/yara             stock CLI (config A plumbing check)
#   oracle/_ref/yarac            stock rules compiler (.yarc fixtures)
#
# The generated parsers (grammar.c, lexer.c, re_*.c, hex_*.c) are checked in
# upstream, so no bison/flex/autotools are needed.

REF ?= /root/reference

# The checked-in parsers must never be regenerated (no yacc/lex here, and a
# fresh checkout may give grammar.y a later mtime than grammar.c).
MAKEFLAGS += -r
.SUFFIXES:
%.c: %.y
%.c: %.l
OUT := oracle/_ref
OBJ := $(OUT)/obj

CC ?= gcc
CFLAGS_REF := -O3 -fPIC -D_GNU_SOURCE -DUSE_LINUX_PROC -DBUCKETS_128=1 \
              -DCHECKSUM_1B=1 -DNDEBUG -w \
              -I$(REF)/libyara/include -I$(REF)/libyara

CORE := ahocorasick arena atoms base64 bitmask compiler endian exec exefiles \
        filemap hash hex_grammar hex_lexer lexer grammar libyara mem modules \
        notebook object parser proc re re_grammar re_lexer rules scan scanner \
        simple_str sizedstr stack stopwatch stream strutils threading
MODS := modules/tests/tests modules/elf/elf modules/math/math modules/time/time \
        modules/pe/pe modules/pe/pe_utils modules/console/console
OTHER := proc/linux tlshc/tlsh tlshc/tlsh_impl tlshc/tlsh_util

SRCS := $(CORE) $(MODS) $(OTHER)
OBJS := $(patsubst %,$(OBJ)/%.o,$(subst /,_,$(SRCS)))

CLI := args common threading yara

HOOKED_OBJS := $(filter-out $(OBJ)/scanner.o,$(OBJS)) $(OBJ)/scanner_hooked.o $(OBJ)/refhook.o

all: $(OUT)/libyara_ref.so $(OUT)/libyara_ref_hooked.so $(OUT)/yara $(OUT)/yarac $(OUT)/refdump \
     $(OUT)/librefmt.so

define OBJ_RULE
$(OBJ)/$(subst /,_,$(1)).o: $(REF)/libyara/$(1).c | $(OBJ)
	$$(CC) $$(CFLAGS_REF) -c $$< -o $$@
endef
$(foreach s,$(SRCS),$(eval $(call OBJ_RULE,$(s))))

$(OBJ):
	mkdir -p $(OBJ)

# Second compile of the reference scanner.c: identical code, but its calls to
# yr_scan_verify_match go through oracle/refhook.c (recorded, then forwarded).
$(OBJ)/scanner_hooked.o: $(REF)/libyara/scanner.c | $(OBJ)
	$(CC) $(CFLAGS_REF) -Dyr_scan_verify_match=yr_refhook_verify_match -c $< -o $@

$(OBJ)/refhook.o: oracle/refhook.c | $(OBJ)
	$(CC) $(CFLAGS_REF) -c $< -o $@

$(OUT)/libyara_ref_hooked.so: $(HOOKED_OBJS)
	$(CC) -shared -o $@ $(HOOKED_OBJS) -lpthread -lm

$(OUT)/refdump: oracle/refdump.c $(OUT)/libyara_ref_hooked.so
	$(CC) -O2 -D_GNU_SOURCE -Wall -I$(REF)/libyara/include -I$(REF)/libyara $< -o $@ \
	  -L$(OUT) -lyara_ref_hooked -Wl,-rpath,'$$ORIGIN' -lpthread -lm

# stock libyara, one scanner per thread over contiguous slices (bench.py's
# multi-threaded CPU baseline)
$(OUT)/librefmt.so: oracle/refmt.c $(OUT)/libyara_ref.so
	$(CC) -O2 -fPIC -shared -D_GNU_SOURCE -Wall -I$(REF)/libyara/include -I$(REF)/libyara $< -o $@ \
	  -L$(OUT) -lyara_ref -Wl,-rpath,'$$ORIGIN' -lpthread -lm

$(OUT)/libyara_ref.so: $(OBJS)
	$(CC) -shared -o $@ $(OBJS) -lpthread -lm

$(OUT)/yara: $(OUT)/libyara_ref.so $(patsubst %,$(REF)/cli/%.c,$(CLI))
	$(CC) -O2 -D_GNU_SOURCE -w -I$(REF)/libyara/include -I$(REF)/cli -I$(REF) \
	  $(patsubst %,$(REF)/cli/%.c,$(CLI)) -o $@ -L$(OUT) -lyara_ref \
	  -Wl,-rpath,'$$ORIGIN' -lpthread -lm

# stock rules compiler: writes the .yarc fixtures of tests/golden/yarc/
$(OUT)/yarac: $(OUT)/libyara_ref.so $(REF)/cli/yarac.c $(REF)/cli/args.c $(REF)/cli/common.c
	$(CC) -O2 -D_GNU_SOURCE -w -I$(REF)/libyara/include -I$(REF)/cli -I$(REF) \
	  $(REF)/cli/yarac.c $(REF)/cli/args.c $(REF)/cli/common.c -o $@ -L$(OUT) -lyara_ref \
	  -Wl,-rpath,'$$ORIGIN' -lpthread -lm

clean:
	rm -rf $(OUT)
.PHONY: all clean
