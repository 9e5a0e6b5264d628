# libyara built with YR_PROFILING_ENABLED (test infrastructure): the reference
# sources compiled in place, as oracle/ref.mk does, with the profiling counters
# on -- and the integration shim plus its end-to-end checker built against it,
# so tests/test_e2e_libyara.py can compare libyara's per-rule atom_matches
# (scan.c:1077-1083, yr_scanner_get_profiling_info scanner.c:758-829) of a
# stock scan with the GPU scan's (count-only records, yara_amd.h).
#
#   make -f oracle/refprof.mk REF=/root/reference -j8
#
# Outputs (git-ignored; travel to the GPU box):
#   oracle/_ref/libyara_prof.so              stock libyara, -DYR_PROFILING_ENABLED
#   integration/_build/libyara_gpu_prof.so   yr_gpu_scanner.c, same define
#   integration/_build/e2e_check_prof        e2e_check.c, same define
REF ?= /root/reference
MAKEFLAGS += -r
.SUFFIXES:
%.c: %.y
%.c: %.l
OUT := oracle/_ref
OBJ := $(OUT)/objprof
CC ?= gcc
INC := -I$(REF)/libyara/include -I$(REF)/libyara
DEFS := -DYR_PROFILING_ENABLED
CFLAGS_REF := -O3 -fPIC -D_GNU_SOURCE -DUSE_LINUX_PROC -DBUCKETS_128=1 -DCHECKSUM_1B=1 \
              -DNDEBUG -w $(DEFS) $(INC)

CORE := ahocorasick arena atoms base64 bitmask compiler endian exec exefiles \
        filemap hash hex_grammar hex_lexer lexer grammar libyara mem modules \
        notebook object parser proc re re_grammar re_lexer rules scan scanner \
        simple_str sizedstr stack stopwatch stream strutils threading
MODS := modules/tests/tests modules/elf/elf modules/math/math modules/time/time \
        modules/pe/pe modules/pe/pe_utils modules/console/console
OTHER := proc/linux tlshc/tlsh tlshc/tlsh_impl tlshc/tlsh_util
SRCS := $(CORE) $(MODS) $(OTHER)
OBJS := $(patsubst %,$(OBJ)/%.o,$(subst /,_,$(SRCS)))

all: $(OUT)/libyara_prof.so integration/_build/libyara_gpu_prof.so \
     integration/_build/e2e_check_prof

define OBJ_RULE
$(OBJ)/$(subst /,_,$(1)).o: $(REF)/libyara/$(1).c
	@mkdir -p $(OBJ)
	$$(CC) $$(CFLAGS_REF) -c $$< -o $$@
endef
$(foreach s,$(SRCS),$(eval $(call OBJ_RULE,$(s))))

$(OUT)/libyara_prof.so: $(OBJS)
	$(CC) -shared -o $@ $(OBJS) -lpthread -lm

PROF_LIBS := -L$(OUT) -lyara_prof -Lyara_amd -lyara_amd \
             -Wl,-rpath,'$$ORIGIN/../../oracle/_ref' -Wl,-rpath,'$$ORIGIN/../../yara_amd' \
             -Wl,-rpath,'$$ORIGIN'

integration/_build/libyara_gpu_prof.so: integration/yr_gpu_scanner.c integration/yr_gpu_scanner.h \
                                        $(OUT)/libyara_prof.so include/yara_amd.h
	@mkdir -p integration/_build
	$(CC) -O2 -D_GNU_SOURCE -Wall -Wno-unused-function -fPIC $(DEFS) $(INC) \
	  -shared -o $@ integration/yr_gpu_scanner.c $(PROF_LIBS)

integration/_build/e2e_check_prof: integration/e2e_check.c integration/_build/libyara_gpu_prof.so
	$(CC) -O2 -D_GNU_SOURCE -Wall -Wno-unused-function $(DEFS) $(INC) -o $@ integration/e2e_check.c \
	  -Lintegration/_build -lyara_gpu_prof $(PROF_LIBS) -lpthread -lm
.PHONY: all
