# Sanitizer build of the host code (included by the Makefile when SAN is set; never used on the
# GPU box). Every host translation unit goes through clang (the same compiler as hipcc's host
# side, so one sanitizer runtime): the device plugin's .cpp files and the host part of
# pathtrace.hip get the -fsanitize flags (device code is compiled as usual: host-only
# instrumentation), the front end is compiled with clang++ instead of g++. The libraries use
# the shared sanitizer runtime that the driver executable (tests/native/san_driver.cpp) loads.
comma := ,
.DEFAULT_GOAL := all
SANCXX   := /opt/rocm/llvm/bin/clang++
SANFLAGS := -fsanitize=$(SAN) -fno-omit-frame-pointer -g -fno-sanitize-recover=all
CXX      := $(SANCXX)
EXTRA    += $(SANFLAGS)
HIPEXTRA += $(foreach f,$(subst $(comma), ,$(SAN)),-Xarch_host -fsanitize=$(f)) -fno-gpu-sanitize
SANRT    := $(shell $(SANCXX) -print-resource-dir)/lib/linux
DEVLDFLAGS := -shared-libsan -fsanitize=$(SAN) -Wl,-rpath,$(SANRT)
FELDFLAGS  := -shared-libsan -fsanitize=$(SAN) -Wl,-rpath,$(SANRT) -lz

san: $(LIB)/san_driver $(LIB)/liboracle_san.so

# the oracle, instrumented, linked into the driver (scenes mode renders thumbnails with it)
$(LIB)/liboracle_san.so: ../oracle/yrt_oracle.c ../oracle/yrt_oracle.h
	@mkdir -p $(LIB)
	$(SANCXX) -x c -std=c11 -O1 -fPIC -ffp-contract=off -mfma $(SANFLAGS) -shared-libsan -shared -o $@ $< -lm -lpthread

$(LIB)/san_driver: ../tests/native/san_driver.cpp $(LIB)/libYulioRT_mi355x.so $(LIB)/liboracle_san.so
	$(SANCXX) -std=c++17 -O1 $(SANFLAGS) -shared-libsan -o $@ $< -L$(LIB) -lYulioRT_mi355x -ldevice_singleray_mi355x \
	    -loracle_san -lz -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(SANRT) -lpthread

.PHONY: san
