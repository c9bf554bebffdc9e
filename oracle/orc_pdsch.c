/*
 * oracle/orc_pdsch.c -- TEST INFRASTRUCTURE ONLY.
 * CPU restatement of the PDSCH stages around the turbo decoder (filled in stage by stage).
 */
#include "oracle.h"
