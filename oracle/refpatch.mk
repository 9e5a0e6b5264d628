# libyara with integration/libyara-block-scanner.patch applied (test
# infrastructure): the reference sources are patched in a scratch directory
# OUTSIDE the repository (the three patched files; the other headers are
# symlinked; nothing is copied into the repo) and compiled with the patched
# headers first on the include path.
#
#   make -f oracle/refpatch.mk REF=/root/reference
#
# Outputs (git-ignored; travel to the GPU box):
#   oracle/_ref/libyara_patched.so          stock libyara + the patch
#   integration/_build/libyara_gpu_hook.so  yr_gpu_scanner.c -DYR_HAVE_BLOCK_SCANNER
#   integration/_build/e2e_check_hook       e2e_check.c -DE2E_BLOCK_SCANNER: the GPU
#                                           side through libyara's own entry points
REF ?= /root/reference
MAKEFLAGS += -r
.SUFFIXES:
%.c: %.y
%.c: %.l

PATCH := integration/libyara-block-scanner.patch
SCRATCH ?= $(or $(TMPDIR),/tmp)/yara_amd_refpatch
OUT := oracle/_ref
OBJ := $(OUT)/objp
CC ?= gcc
INC := -I$(SCRATCH)/libyara/include -I$(REF)/libyara/include -I$(REF)/libyara
CFLAGS_REF := -O3 -fPIC -D_GNU_SOURCE -DUSE_LINUX_PROC -DBUCKETS_128=1 -DCHECKSUM_1B=1 \
              -DNDEBUG -w $(INC)

CORE := ahocorasick arena atoms base64 bitmask compiler endian exec exefiles \
        filemap hash hex_grammar hex_lexer lexer grammar libyara mem modules \
        notebook object parser proc re re_grammar re_lexer rules scan \
        simple_str sizedstr stack stopwatch stream strutils threading
MODS := modules/tests/tests modules/elf/elf modules/math/math modules/time/time \
        modules/pe/pe modules/pe/pe_utils modules/console/console
OTHER := proc/linux tlshc/tlsh tlshc/tlsh_impl tlshc/tlsh_util
SRCS := $(CORE) $(MODS) $(OTHER)
OBJS := $(patsubst %,$(OBJ)/%.o,$(subst /,_,$(SRCS))) $(OBJ)/scanner.o

all: $(OUT)/libyara_patched.so integration/_build/libyara_gpu_hook.so \
     integration/_build/e2e_check_hook

$(SCRATCH)/.stamp: $(PATCH) oracle/refpatch.mk
	rm -rf $(SCRATCH)
	mkdir -p $(SCRATCH)/libyara/include/yara
	cp $(REF)/libyara/scanner.c $(SCRATCH)/libyara/
	cp $(REF)/libyara/include/yara/types.h $(REF)/libyara/include/yara/scanner.h \
	   $(SCRATCH)/libyara/include/yara/
	patch -s -d $(SCRATCH) -p1 < $(PATCH)
	# the other headers of include/yara/ as symlinks, so the patched ones'
	# quoted includes ("notebook.h") resolve next to them
	for h in $(REF)/libyara/include/yara/*.h; do \
	  [ -e $(SCRATCH)/libyara/include/yara/$$(basename $$h) ] || ln -s $$h $(SCRATCH)/libyara/include/yara/; \
	done
	touch $@

define OBJ_RULE
$(OBJ)/$(subst /,_,$(1)).o: $(REF)/libyara/$(1).c $(SCRATCH)/.stamp
	@mkdir -p $(OBJ)
	$$(CC) $$(CFLAGS_REF) -c $$< -o $$@
endef
$(foreach s,$(SRCS),$(eval $(call OBJ_RULE,$(s))))

$(OBJ)/scanner.o: $(SCRATCH)/.stamp
	@mkdir -p $(OBJ)
	$(CC) $(CFLAGS_REF) -c $(SCRATCH)/libyara/scanner.c -o $@

$(OUT)/libyara_patched.so: $(OBJS)
	$(CC) -shared -o $@ $(OBJS) -lpthread -lm

HOOK_LIBS := -L$(OUT) -lyara_patched -Lyara_amd -lyara_amd \
             -Wl,-rpath,'$$ORIGIN/../../oracle/_ref' -Wl,-rpath,'$$ORIGIN/../../yara_amd' \
             -Wl,-rpath,'$$ORIGIN'

integration/_build/libyara_gpu_hook.so: integration/yr_gpu_scanner.c integration/yr_gpu_scanner.h \
                                        $(OUT)/libyara_patched.so include/yara_amd.h
	@mkdir -p integration/_build
	$(CC) -O2 -D_GNU_SOURCE -Wall -Wno-unused-function -fPIC -DYR_HAVE_BLOCK_SCANNER $(INC) \
	  -shared -o $@ integration/yr_gpu_scanner.c $(HOOK_LIBS)

integration/_build/e2e_check_hook: integration/e2e_check.c integration/_build/libyara_gpu_hook.so
	$(CC) -O2 -D_GNU_SOURCE -Wall -Wno-unused-function -DYR_HAVE_BLOCK_SCANNER -DE2E_BLOCK_SCANNER \
	  $(INC) -o $@ integration/e2e_check.c -Lintegration/_build -lyara_gpu_hook $(HOOK_LIBS) -lpthread -lm

.PHONY: all
