# Builds the gfx950 HIP library of the YOLOv11 inference path in-tree.
#   make            -> yolo-infer-pt_amd/yolo_hip/libyolo_hip.so
#   make oracle     -> oracle/_c/liboracle_nms.so (CPU checker, tests only)
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
ARCH ?= gfx950
PKG := yolo-infer-pt_amd
SRC := $(PKG)/csrc
OUT ?= $(PKG)/yolo_hip/libyolo_hip.so
OBJDIR ?= build/obj
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Iinclude -I$(SRC) \
            -fhip-fp32-correctly-rounded-divide-sqrt -Wno-unused-result $(EXTRA)
OBJS := $(OBJDIR)/engine.o $(OBJDIR)/conv.o $(OBJDIR)/misc.o $(OBJDIR)/nms.o $(OBJDIR)/conv_mx.o $(OBJDIR)/nms_host.o \
        $(OBJDIR)/preprocess.o $(OBJDIR)/head.o $(OBJDIR)/c3k2.o $(OBJDIR)/conv_rw.o $(OBJDIR)/c3k.o $(OBJDIR)/boxc.o $(OBJDIR)/pwchain.o

all: $(OUT)

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/engine.o: $(SRC)/engine.cpp $(SRC)/common.h $(SRC)/conv_mx.h include/yolo_hip.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/conv.o: $(SRC)/conv.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/misc.o: $(SRC)/misc.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/conv_mx.o: $(SRC)/conv_mx.hip $(SRC)/conv_mx.h $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/conv_rw.o: $(SRC)/conv_rw.hip $(SRC)/conv_mx.h $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/nms_host.o: $(SRC)/nms_host.cpp include/yolo_hip.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(OBJDIR)/head.o: $(SRC)/head.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/c3k2.o: $(SRC)/c3k2.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/c3k.o: $(SRC)/c3k.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/boxc.o: $(SRC)/boxc.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/pwchain.o: $(SRC)/pwchain.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/preprocess.o: $(SRC)/preprocess.hip $(SRC)/common.h include/yolo_hip.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -ffp-contract=off -c $< -o $@

$(OBJDIR)/nms.o: $(SRC)/nms.hip $(SRC)/common.h $(SRC)/dtypes.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -ffp-contract=off -c $< -o $@

$(OUT): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(OUT)

.PHONY: all clean
