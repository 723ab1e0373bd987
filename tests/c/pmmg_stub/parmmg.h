/*
 * parmmg.h -- TEST-LOCAL declarations for compiling integration/pmmg_pmx.c
 * outside a ParMmg build (tests/c/adapter_demo.c).
 *
 * This is NOT the reference's header: it declares only the handful of
 * ParMmg / Mmg structure fields and helpers the adapter touches, with the
 * reference's names (src/libparmmgtypes.h, src/parmmg.h, Mmg's
 * libmmgtypes.h) so that the adapter source compiles unchanged in both
 * places.  Layouts are not Mmg's: the adapter reads the records through
 * strides and field addresses only, which is what the test exercises.
 * MPI is absent: the test runs one rank (nprocs = 1).  The Mmg/ParMmg helper
 * functions declared at the end are implemented by the test driver
 * (recording what the adapter hands them).
 */
#ifndef PMX_TEST_PARMMG_H
#define PMX_TEST_PARMMG_H
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* --- Mmg ------------------------------------------------------------------ */
#define MG_GEO    ((int16_t)1 << 1)
#define MG_REQ    ((int16_t)1 << 2)
#define MG_BDY    ((int16_t)1 << 4)
#define MG_NUL    ((int16_t)1 << 14)
#define MG_NOM    ((int16_t)1 << 3)
#define MG_CRN    ((int16_t)1 << 5)
#define MG_EOK(pt) (pt && ((pt)->v[0] > 0))

typedef struct {
  double   c[3];
  double   n[3];
  int      ref, xp, tmp, flag, s;
  uint16_t tag;
  int8_t   tagdel;
} MMG5_Point;
typedef MMG5_Point *MMG5_pPoint;

typedef struct {
  double  qual;
  int     v[4];
  int     ref, base, mark, xt, flag;
  int16_t tag;
} MMG5_Tetra;
typedef MMG5_Tetra *MMG5_pTetra;

typedef struct {
  double  qual;
  int     v[3], ref, base, cc, edg[3], flag;
  int16_t tag[3];
} MMG5_Tria;
typedef MMG5_Tria *MMG5_pTria;

typedef struct {
  int     a, b, ref, base;
  int16_t tag;
} MMG5_Edge;
typedef MMG5_Edge *MMG5_pEdge;

typedef struct {
  int      ref[4], edg[6];
  int16_t  ftag[4];
  uint16_t tag[6];
  int8_t   ori;
} MMG5_xTetra;
typedef MMG5_xTetra *MMG5_pxTetra;

typedef struct {
  double  n1[3], n2[3];
  int8_t  nnor;
} MMG5_xPoint;
typedef MMG5_xPoint *MMG5_pxPoint;

typedef struct {
  double  hsiz, hausd;
  int     imprim, renum;
  int8_t  optimLES;
} MMG5_Info;

typedef struct {
  int         np, ne, nt, na, nsols, base;
  int         xt, xp;                  /* xTetra / xPoint counts */
  MMG5_pPoint point;
  MMG5_pTetra tetra;
  MMG5_pxTetra xtetra;
  MMG5_pxPoint xpoint;
  MMG5_pTria  tria;
  MMG5_pEdge  edge;
  int        *adja, *adjt;
  MMG5_Info   info;
} MMG5_Mesh;
typedef MMG5_Mesh *MMG5_pMesh;

typedef struct {
  int     np, size;
  double *m;
} MMG5_Sol;
typedef MMG5_Sol *MMG5_pSol;

typedef struct {
  void *geom;
} MMG5_HGeom;

#define MMG5_DEL_MEM(mesh, p) do { free(p); (p) = NULL; } while (0)

/* --- ParMmg --------------------------------------------------------------- */
#define PMMG_SUCCESS      0
#define PMMG_INQUA        1
#define PMMG_OUTQUA       2
#define PMMG_QUAL_HISSIZE 5
#define PMMG_VERB_VERSION 0

typedef int MPI_Comm;

typedef struct {
  int     nitem;
  int    *intvalues;
} PMMG_Int_comm;
typedef PMMG_Int_comm *PMMG_pInt_comm;

typedef struct {
  int  color_in, color_out;
  int *int_comm_index;
  int  nitem;
} PMMG_Ext_comm;
typedef PMMG_Ext_comm *PMMG_pExt_comm;

typedef struct {
  MMG5_pMesh mesh;
  MMG5_pSol  met;
  MMG5_pSol  field;
  int        nitem_int_node_comm;
  int       *node2int_node_comm_index1, *node2int_node_comm_index2;
  int        nitem_int_edge_comm;
  int       *edge2int_edge_comm_index1, *edge2int_edge_comm_index2;
} PMMG_Grp;
typedef PMMG_Grp *PMMG_pGrp;

typedef struct {
  int     imprim, imprim0, root;
  uint8_t inputMet;
} PMMG_Info;

typedef struct {
  MPI_Comm       comm;
  int            myrank, nprocs, ngrp;
  PMMG_pGrp      listgrp, old_listgrp;
  PMMG_Info      info;
  PMMG_pInt_comm int_node_comm, int_edge_comm;
  int            next_node_comm, next_edge_comm;
  PMMG_pExt_comm ext_node_comm, ext_edge_comm;
} PMMG_ParMesh;
typedef PMMG_ParMesh *PMMG_pParMesh;

/* memory accounting macros (src/parmmg.h:300-406): plain calloc/free here */
#define PMMG_CALLOC(parmesh, ptr, n, type, msg, on_failure) \
  do { (ptr) = (type *)calloc((size_t)(n) > 0 ? (size_t)(n) : 1, sizeof(type)); \
       if (!(ptr)) { on_failure; } } while (0)
#define PMMG_MALLOC(parmesh, ptr, n, type, msg, on_failure) \
  do { (ptr) = (type *)malloc(((size_t)(n) > 0 ? (size_t)(n) : 1) * sizeof(type)); \
       if (!(ptr)) { on_failure; } } while (0)
#define PMMG_DEL_MEM(parmesh, ptr, type, msg) do { free(ptr); (ptr) = NULL; } while (0)

/* the seams (src/parmmg.h:472-473,564-566), defined by integration/pmmg_pmx.c */
int PMMG_interpMetricsAndFields(PMMG_pParMesh parmesh, int *permNodGlob);
int PMMG_copyMetricsAndFields_point(MMG5_pMesh mesh, MMG5_pMesh oldMesh, MMG5_pSol met, MMG5_pSol oldMet,
                                    MMG5_pSol field, MMG5_pSol oldField, int *permNodGlob, uint8_t inputMet);
int PMMG_qualhisto(PMMG_pParMesh parmesh, int opt, int isCentral);
int PMMG_prilen(PMMG_pParMesh parmesh, int8_t metRidTyp, int isCentral);
int PMMG_tetraQual(PMMG_pParMesh parmesh, int8_t metRidTyp);

/* helpers the adapter calls, implemented by the test driver */
int  MMG3D_displayQualHisto_internal(int64_t ne, double max, double avg, double min, int iel, int good,
                                     int med, int his[PMMG_QUAL_HISSIZE], int nrid, int optimLES,
                                     int imprim);
int  MMG5_displayLengthHisto_internal(int ned, int amin, int bmin, double lmin, int amax, int bmax,
                                      double lmax, int nullEdge, double *bd, int *hl, int8_t shift,
                                      int imprim);
int  PMMG_hashPar(MMG5_pMesh mesh, MMG5_HGeom *pHash);
int  MMG5_hGet(MMG5_HGeom *hash, int a, int b, int *ref, int16_t *tag);
int  PMMG_build_edgeComm(PMMG_pParMesh parmesh, MMG5_pMesh mesh, MMG5_HGeom *hpar);
void PMMG_edge_comm_free(PMMG_pParMesh parmesh);
/* the adapter's MPI calls (the RCCL id's broadcast, the ranks' agreement on
 * their local results): implemented by the test driver (never reached with
 * one rank; a socketpair shim for the two-process driver) */
int  MPI_Bcast(void *buf, int count, int type, int root, MPI_Comm comm);
int  MPI_Allreduce(const void *sendbuf, void *recvbuf, int count, int type, int op, MPI_Comm comm);
#define MPI_BYTE 1
#define MPI_INT 2
#define MPI_MIN 1
#define MPI_IN_PLACE ((void *)1)

#endif
